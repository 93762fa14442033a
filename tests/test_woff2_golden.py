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
