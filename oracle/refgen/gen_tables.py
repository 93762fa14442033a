#!/usr/bin/env python3
"""Generate the RFC 7932 constant data (static dictionary, 121 word transforms, literal
context lookup) as C headers for the oracle and the product.

These are RFC 7932 Appendix A/B and section 7.1 data, not code.  They are extracted here
from the reference's packed representation (/root/reference/src/decode/engine.ts,
dictionary-bin.ts) and cross-checked against independent sources available in this
container:
  * the dictionary blob is decoded with Node's bundled native brotli 1.0.9 (zlib) AND with
    the type-erased reference decoder; both must agree;
  * the decoder's context LUT (engine.ts:1937-1969) must equal the encoder's
    CONTEXT_LOOKUP_TABLE (src/encode/context.ts:12) mode by mode.

Outputs (committed):
  brotli-lib_amd/data/dictionary.bin         122,784 bytes
  brotli-lib_amd/csrc/rfc_tables.h           transforms + context LUT + dictionary offsets
  brotli-lib_amd/csrc/rfc_dictionary.inc     dictionary bytes as a C initializer list
  oracle/rfc_tables.h, oracle/rfc_dictionary.inc   identical copies for the oracle
"""
import hashlib
import os
import re
import subprocess
import sys

REF = '/root/reference'
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def js_string_literal(s):
    """decode a double-quoted JS string body (escapes used in engine.ts)."""
    out = []
    i = 0
    while i < len(s):
        c = s[i]
        if c == '\\':
            n = s[i + 1]
            if n == 'x':
                out.append(chr(int(s[i + 2:i + 4], 16)))
                i += 4
                continue
            out.append({'n': '\n', 't': '\t', 'r': '\r', '"': '"', "'": "'", '\\': '\\'}[n])
            i += 2
            continue
        out.append(c)
        i += 1
    return ''.join(out)


def main():
    eng = open(os.path.join(REF, 'src/decode/engine.ts'), encoding='utf-8').read()
    m = re.search(r'unpackTransforms\(RFC_TRANSFORMS\.prefixSuffixStorage, RFC_TRANSFORMS\.prefixSuffixHeads, '
                  r'RFC_TRANSFORMS\.triplets, "((?:[^"\\]|\\.)*)", "((?:[^"\\]|\\.)*)"\);', eng)
    prefix_suffix_src = js_string_literal(m.group(1))
    transforms_src = js_string_literal(m.group(2))
    # engine.ts:1535-1551
    storage, heads = [], [0]
    for ch in prefix_suffix_src:
        c = ord(ch)
        if c == 35:
            heads.append(len(storage))
        else:
            storage.append(c)
    assert len(heads) == 51 and len(storage) == 167, (len(heads), len(storage))
    triplets = [ord(transforms_src[i]) - 32 for i in range(363)]
    assert len(triplets) == 363

    m = re.search(r'unpackLookupTable\(LOOKUP, "((?:[^"\\]|\\.)*)", "((?:[^"\\]|\\.)*)"\);', eng)
    utf_map, utf_rle = js_string_literal(m.group(1)), js_string_literal(m.group(2))
    lut = [0] * 2048   # engine.ts:1937-1969
    for i in range(256):
        lut[i] = i & 0x3F
        lut[512 + i] = i >> 2
        lut[1792 + i] = 2 + (i >> 6)
    for i in range(128):
        lut[1024 + i] = 4 * (ord(utf_map[i]) - 32)
    for i in range(64):
        lut[1152 + i] = i & 1
        lut[1216 + i] = 2 + (i & 1)
    off = 1280
    for k in range(19):
        for _ in range(ord(utf_rle[k]) - 32):
            lut[off] = k & 3
            off += 1
    for i in range(16):
        lut[1792 + i] = 1
        lut[2032 + i] = 6
    lut[1792] = 0
    lut[2047] = 7
    for i in range(256):
        lut[1536 + i] = lut[1792 + i] << 3

    ctx = open(os.path.join(REF, 'src/encode/context.ts'), encoding='utf-8').read()
    body = re.search(r'CONTEXT_LOOKUP_TABLE = new Uint8Array\(\[(.*?)\]\)', ctx, re.S).group(1)
    body = re.sub(r'//[^\n]*', '', body)
    enc_lut = [int(x) for x in re.findall(r'\d+', body)]
    assert len(enc_lut) == 2048
    assert enc_lut == lut, 'encoder/decoder context LUT disagree'

    # static dictionary: decode the reference's compressed blob two independent ways
    blob_src = open(os.path.join(REF, 'src/decode/dictionary-bin.ts'), encoding='utf-8').read()
    b64 = re.search(r'compressedDictionary = "([^"]+)"', blob_src).group(1)
    import base64
    comp = base64.b64decode(b64)
    native = subprocess.run(['node', '-e',
                             'const z=require("zlib");process.stdout.write(z.brotliDecompressSync(Buffer.from(process.argv[1],"base64")))',
                             b64], capture_output=True, check=True).stdout
    assert len(native) == 122784, len(native)
    erased = os.path.join(ROOT, 'oracle/_ref/asis/src/decode/decode.mjs')
    if os.path.exists(erased):
        ref_out = subprocess.run(['node', '--input-type=module', '-e',
                                  'import {brotliDecode} from "%s";' % erased +
                                  'process.stdout.write(Buffer.from(brotliDecode(Buffer.from(process.argv[1],"base64"))))',
                                  b64], capture_output=True, check=True).stdout
        assert ref_out == native, 'reference and native brotli disagree on the dictionary'
    sha = hashlib.sha256(native).hexdigest()

    # word offsets per length (dictionary.ts:34-46 / RFC 7932 appendix A)
    size_bits = [0, 0, 0, 0, 10, 10, 11, 11, 10, 10, 10, 10, 10, 9, 9, 8, 7, 7, 8, 7, 7, 6, 6, 5, 5]
    offsets, pos = [], 0
    for i, b in enumerate(size_bits):
        offsets.append(pos)
        if b:
            pos += i << b
    assert pos == 122784
    offsets += [pos] * (32 - len(offsets))
    size_bits += [0] * (32 - len(size_bits))

    # fast-log.ts:6-93 kLog2Table (upstream brotli fast_log.c): NOT correctly rounded log2,
    # so the exact doubles are carried over (as hex floats) for bit-exact cost models.
    fl = open(os.path.join(REF, 'src/encode/fast-log.ts'), encoding='utf-8').read()
    lbody = re.search(r'kLog2Table = new Float64Array\(\[(.*?)\]\)', fl, re.S).group(1)
    log2_table = [float(x) for x in re.findall(r'[\d.]+', lbody)]
    assert len(log2_table) == 256

    def carr(name, ctype, vals, per=16):
        lines = []
        for i in range(0, len(vals), per):
            lines.append('  ' + ', '.join(str(v) for v in vals[i:i + per]) + ',')
        return 'RFC_CONST %s %s[%d] = {\n%s\n};\n' % (ctype, name, len(vals), '\n'.join(lines))

    hdr = ['/* GENERATED by oracle/refgen/gen_tables.py -- RFC 7932 constant data. Do not edit. */',
           '#ifndef BROTLI_RFC_TABLES_H_', '#define BROTLI_RFC_TABLES_H_', '#include <stdint.h>', '',
           '/* storage class of every table; HIP device code defines it as `static __device__ const` */',
           '#ifndef RFC_CONST', '#define RFC_CONST static const', '#endif', '',
           '#define RFC_DICT_SIZE 122784',
           '#define RFC_DICT_SHA256 "%s"' % sha,
           '#define RFC_NUM_TRANSFORMS 121', '',
           '/* RFC 7932 appendix B: prefix/suffix strings ("#"-separated heads) and (prefix, type, suffix) triplets */',
           carr('kRfcPrefixSuffix', 'uint8_t', storage),
           carr('kRfcPrefixSuffixHeads', 'uint16_t', heads),
           carr('kRfcTransformTriplets', 'uint8_t', triplets, 21),
           '/* RFC 7932 section 7.1 literal context lookup: [mode*512 + p1] | [mode*512 + 256 + p2] */',
           carr('kRfcContextLut', 'uint8_t', lut, 32),
           '/* encoder cost-model table (fast-log.ts:6-93), exact doubles */',
           'RFC_CONST double kFastLog2Table[256] = {\n%s\n};\n' % '\n'.join(
               '  ' + ', '.join(float.hex(v) for v in log2_table[i:i + 4]) + ',' for i in range(0, 256, 4)),
           '/* RFC 7932 appendix A: NDBITS per word length and word-list offsets */',
           carr('kRfcDictSizeBits', 'uint8_t', size_bits, 32),
           carr('kRfcDictOffsets', 'uint32_t', offsets, 8),
           '#endif', '']
    hdr = '\n'.join(hdr)
    inc = '/* GENERATED by oracle/refgen/gen_tables.py: RFC 7932 static dictionary bytes (sha256 %s) */\n' % sha
    inc += '\n'.join(','.join(str(b) for b in native[i:i + 40]) + ',' for i in range(0, len(native), 40)) + '\n'

    os.makedirs(os.path.join(ROOT, 'brotli-lib_amd/data'), exist_ok=True)
    with open(os.path.join(ROOT, 'brotli-lib_amd/data/dictionary.bin'), 'wb') as f:
        f.write(native)
    for d in ('brotli-lib_amd/csrc', 'oracle'):
        with open(os.path.join(ROOT, d, 'rfc_tables.h'), 'w') as f:
            f.write(hdr)
        with open(os.path.join(ROOT, d, 'rfc_dictionary.inc'), 'w') as f:
            f.write(inc)
    print('dictionary sha256', sha, 'transforms', len(triplets) // 3, 'lut ok')


if __name__ == '__main__':
    sys.exit(main())
