"""Goldens for the GPU WOFF2 'glyf' and 'hmtx' transforms: fontTools' WOFF2GlyfTable /
WOFF2HmtxTable.transform of the reference's TrueType bench fonts (enc-ttf.bin, and
enc-var-ttf decoded from its .br by the oracle), and for hmtx also of byte-edited variants
whose side bearings differ from xMin (hmtx_variants).  Writes glyf_golden.json and
hmtx_golden.json (sizes, sha256).  Run on the CPU:
    python3 tests/golden/woff2/make_golden.py"""
import hashlib
import io
import json
import os
import struct
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
TESTS = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, TESTS)


def fonts():
    import _oracle
    bench = os.path.join(TESTS, 'golden', 'bench')
    with open(os.path.join(bench, 'enc-ttf.bin'), 'rb') as f:
        yield 'enc-ttf', f.read()
    with open(os.path.join(bench, 'enc-var-ttf.br'), 'rb') as f:
        yield 'enc-var-ttf', _oracle.decode(f.read())


def transform(ttf):
    from fontTools.ttLib import TTFont
    from fontTools.ttLib.woff2 import WOFF2GlyfTable
    font = TTFont(io.BytesIO(ttf))
    t = WOFF2GlyfTable()
    t.__dict__.update(font['glyf'].__dict__)
    return t.transform(font)


def _table(ttf, tag):
    n = struct.unpack('>H', ttf[4:6])[0]
    for i in range(n):
        r = ttf[12 + 16 * i:28 + 16 * i]
        if r[:4] == tag:
            return struct.unpack('>LL', r[8:16])
    raise KeyError(tag)


def hmtx_variants(ttf):
    """(tag, font bytes): as is; a proportional glyph's lsb moved off its xMin; the last
    (monospaced) glyph's; both (no transform applies)."""
    hoff, _ = _table(ttf, b'hmtx')
    hh, _ = _table(ttf, b'hhea')
    mp, _ = _table(ttf, b'maxp')
    nhm = struct.unpack('>H', ttf[hh + 34:hh + 36])[0]
    ng = struct.unpack('>H', ttf[mp + 4:mp + 6])[0]

    def bump(b, at):
        v = struct.unpack('>h', b[at:at + 2])[0]
        b[at:at + 2] = struct.pack('>h', v + 1 if v < 32767 else v - 1)

    prop_at = hoff + 4 * 5 + 2
    mono_at = hoff + 4 * nhm + 2 * (ng - 1 - nhm) if ng > nhm else None
    yield 'asis', bytes(ttf)
    b = bytearray(ttf)
    bump(b, prop_at)
    yield 'prop', bytes(b)
    if mono_at is not None:
        b = bytearray(ttf)
        bump(b, mono_at)
        yield 'mono', bytes(b)
        b = bytearray(ttf)
        bump(b, prop_at)
        bump(b, mono_at)
        yield 'both', bytes(b)


def transform_hmtx(ttf):
    from fontTools.ttLib import TTFont
    from fontTools.ttLib.woff2 import WOFF2HmtxTable
    font = TTFont(io.BytesIO(ttf))
    t = WOFF2HmtxTable()
    t.__dict__.update(font['hmtx'].__dict__)
    return t.transform(font)


def main():
    out = {}
    for name, ttf in fonts():
        data = transform(ttf)
        hdr = struct.unpack('>HHHHLLLLLLL', data[:36])
        out[name] = {'ttf_sha256': hashlib.sha256(ttf).hexdigest(), 'size': len(data),
                     'sha256': hashlib.sha256(data).hexdigest(), 'header': list(hdr)}
    with open(os.path.join(HERE, 'glyf_golden.json'), 'w') as f:
        json.dump({'generator': 'fontTools WOFF2GlyfTable.transform', 'fonts': out}, f, indent=1, sort_keys=True)
    print(json.dumps(out, indent=1))
    hm = {}
    for name, ttf in fonts():
        for tag, v in hmtx_variants(ttf):
            d = transform_hmtx(v)
            hm['%s/%s' % (name, tag)] = None if d is None else {
                'size': len(d), 'flags': d[0], 'sha256': hashlib.sha256(d).hexdigest()}
    with open(os.path.join(HERE, 'hmtx_golden.json'), 'w') as f:
        json.dump({'generator': 'fontTools WOFF2HmtxTable.transform', 'fonts': hm}, f, indent=1, sort_keys=True)
    print(json.dumps(hm, indent=1))


if __name__ == '__main__':
    main()
