"""Goldens for the GPU WOFF2 'glyf' transform: fontTools' WOFF2GlyfTable.transform of the
reference's TrueType bench fonts (enc-ttf.bin, and enc-var-ttf decoded from its .br by the
oracle).  Writes glyf_golden.json (sizes, stream sizes, sha256).  Run on the CPU:
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


if __name__ == '__main__':
    main()
