"""GPU WOFF2 'glyf' transform (brotli-lib_amd/csrc/woff2.hip): byte-exact with
fontTools' WOFF2GlyfTable.transform on the reference's TrueType bench fonts (goldens in
tests/golden/woff2), and the transformed table through the FONT-mode encoder and back."""
import hashlib
import json
import os
import sys

import pytest

import _inputs
import _oracle
import brotli_amd

pytestmark = pytest.mark.gpu
HERE = os.path.join(_inputs.GOLDEN, 'woff2')
sys.path.insert(0, HERE)


def _fonts():
    import make_golden
    return list(make_golden.fonts())


def test_glyf_transform_matches_fonttools():
    with open(os.path.join(HERE, 'glyf_golden.json')) as f:
        gold = json.load(f)['fonts']
    for name, ttf in _fonts():
        got = brotli_amd.woff2_transform_glyf(ttf)
        if hashlib.sha256(got).hexdigest() != gold[name]['sha256']:
            detail = ''
            try:
                import make_golden
                want = make_golden.transform(ttf)
                i = next((k for k in range(min(len(got), len(want))) if got[k] != want[k]), min(len(got), len(want)))
                detail = 'first difference at %d of %d/%d; header got %s want %s' % (
                    i, len(got), len(want), got[:36].hex(), want[:36].hex())
            except ImportError:
                pass
            pytest.fail('%s: transformed glyf differs from fontTools (%s)' % (name, detail))


def test_transformed_glyf_roundtrips_font_mode():
    for name, ttf in _fonts():
        t = brotli_amd.woff2_transform_glyf(ttf)
        enc = brotli_amd.brotliEncode(t, {'quality': 11, 'mode': brotli_amd.EncoderMode.FONT})
        assert _oracle.decode(enc) == t, name
        assert brotli_amd.brotliDecode(enc) == t, name


def test_malformed_fonts_are_rejected():
    ttf = _fonts()[0][1]
    for bad in (b'', ttf[:11], ttf[:200]):
        with pytest.raises(brotli_amd.BrotliError):
            brotli_amd.woff2_transform_glyf(bad)


def test_hmtx_transform_matches_fonttools():
    """WOFF2 section 5.4 on the GPU against fontTools' WOFF2HmtxTable.transform: the bench fonts
    as they are (both side-bearing arrays dropped), with a proportional or the monospaced
    glyph's lsb moved off its xMin (that array kept), and with both (no transform: None)."""
    import make_golden
    with open(os.path.join(HERE, 'hmtx_golden.json')) as f:
        gold = json.load(f)['fonts']
    seen = 0
    for name, ttf in _fonts():
        for tag, v in make_golden.hmtx_variants(ttf):
            want = gold['%s/%s' % (name, tag)]
            got = brotli_amd.woff2_transform_hmtx(v)
            if want is None:
                assert got is None, (name, tag)
            else:
                assert got is not None and got[0] == want['flags'] and len(got) == want['size'], (name, tag)
                assert hashlib.sha256(got).hexdigest() == want['sha256'], (name, tag)
            seen += 1
    assert seen == 8
