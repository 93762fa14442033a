"""The WOFF2 'glyf' goldens (tests/golden/woff2/glyf_golden.json) are fontTools'
WOFF2GlyfTable.transform of the reference's TrueType bench fonts: regenerate and compare."""
import hashlib
import json
import os
import sys

import pytest

import _inputs

HERE = os.path.join(_inputs.GOLDEN, 'woff2')
sys.path.insert(0, HERE)


def test_goldens_are_fonttools_output():
    pytest.importorskip('fontTools')
    import make_golden
    with open(os.path.join(HERE, 'glyf_golden.json')) as f:
        gold = json.load(f)['fonts']
    for name, ttf in make_golden.fonts():
        assert hashlib.sha256(ttf).hexdigest() == gold[name]['ttf_sha256']
        data = make_golden.transform(ttf)
        assert len(data) == gold[name]['size'] and hashlib.sha256(data).hexdigest() == gold[name]['sha256'], name


def test_c3_generator_builds_valid_fonts():
    """datagen.glyf_font (C3's inputs): glyph sets from the reference's Inter bench font,
    jittered per seed, are well-formed TrueType: fontTools' WOFF2 glyf transform accepts them."""
    import pytest
    pytest.importorskip('fontTools')
    import sys, os
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), 'golden', 'woff2'))
    import make_golden
    from brotli_amd import datagen
    a = datagen.glyf_font(1000, 800)
    assert datagen.glyf_font(1000, 800) == a and datagen.glyf_font(1001, 800) != a
    t = make_golden.transform(a)
    assert len(t) > 10000
    s = datagen.glyf_font_stream(65536, 1002, transform=make_golden.transform)
    assert len(s) == 65536
