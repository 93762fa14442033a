#!/usr/bin/env python3
"""Generate tests/golden/decode_compound.json: streams that address a customDictionary
(compound dictionary, engine.ts:142-159,946-1011), decoded by the type-erased reference
itself (run_ref.mjs) with the dictionary passed as Uint8Array and as Int8Array.

TEST INFRASTRUCTURE ONLY.  The streams are written here by a minimal RFC 7932 bit writer
(one metablock, one block type per category, simple prefix codes: two literals, two
command symbols, two distance symbols), with copies whose distances land inside the
output, on the dictionary's tail (distance in (pos, pos + length]), before it (the
reference's -9), and past it into the static dictionary.  The expected output / error of
every stream is the reference's.

usage: python3 oracle/refgen/make_compound.py
"""
import base64
import hashlib
import json
import os
import random
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, 'tests'))
import _inputs  # noqa: E402
RUN = os.path.join(ROOT, 'oracle', 'refgen', 'run_ref.mjs')
OUT = os.path.join(ROOT, 'tests', 'golden', 'decode_compound.json')


class Bits:
    def __init__(self):
        self.v, self.n = 0, 0

    def put(self, nbits, val):
        self.v |= (val & ((1 << nbits) - 1)) << self.n
        self.n += nbits

    def bytes(self):
        return self.v.to_bytes((self.n + 7) // 8, 'little')


INS_BASE = [0, 1, 2, 3, 4, 5, 6, 8, 10, 14, 18, 26, 34, 50, 66, 98, 130, 194, 322, 578, 1090, 2114, 6210, 22594]
INS_EXTRA = [0, 0, 0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 7, 8, 9, 10, 12, 14, 24]
COPY_BASE = [2, 3, 4, 5, 6, 7, 8, 9, 10, 12, 14, 18, 22, 30, 38, 54, 70, 102, 134, 198, 326, 582, 1094, 2118]
COPY_EXTRA = [0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 7, 8, 9, 10, 24]


def combine(ic, cc):   # command symbol with an explicit distance (RFC 7932 section 5)
    off = 2 * ((cc >> 3) + 3 * (ic >> 3))
    off = (off << 5) + 0x40 + ((0x520D40 >> off) & 0xC0)
    return off | (cc & 7) | ((ic & 7) << 3)


def dist_symbol(d):   # NPOSTFIX 0, NDIRECT 0: (symbol, nbits, extra) of distance d (> 0)
    dist = d + 3
    bucket = dist.bit_length() - 2
    prefix = (dist >> bucket) & 1
    offset = (2 + prefix) << bucket
    return 16 + 2 * (bucket - 1) + prefix, bucket, dist - offset


def simple_code(w, alphabet_bits, syms):   # HSKIP 1, NSYM-1, symbols (lengths 1,1 for two)
    w.put(2, 1)
    w.put(2, len(syms) - 1)
    for s in syms:
        w.put(alphabet_bits, s)


def rev2(k):
    return ((k & 1) << 1) | (k >> 1)


def make_stream(rng, dict_len, good):
    # two command shapes: (insert code 8 = 10..13, copy code 10 = 14..17), (insert 2, copy code 14 = 38..53)
    shapes = [(8, 10), (2, 14)]
    cmds = sorted(combine(ic, cc) for ic, cc in shapes)
    for _attempt in range(100):
        prog, pos = [], 0
        for _ in range(rng.randrange(3, 40)):
            ic, cc = shapes[rng.randrange(2)]
            ins = INS_BASE[ic] + rng.randrange(1 << INS_EXTRA[ic])
            cl = COPY_BASE[cc] + rng.randrange(1 << COPY_EXTRA[cc])
            lits = [rng.choice(b'ab') for _ in range(ins)]
            pos += ins
            kind = rng.random()
            if (good and kind < 0.6 and pos >= 1) or (not good and kind < 0.4):
                d = rng.randrange(1, pos + 1)          # into the output
            elif good or kind < 0.7:
                d = pos + cl                           # the dictionary's tail, exactly (the reference's rule)
            elif kind < 0.85:
                d = pos + cl + rng.randrange(1, 50)    # before the tail
            else:
                d = pos + rng.randrange(1, cl)         # past the dictionary's end
            prog.append((combine(ic, cc), ic, ins, cc, cl, lits, d))
            pos += cl
        dsyms = sorted(set(dist_symbol(p[6])[0] for p in prog))
        if len(dsyms) <= 4:
            break
    else:
        raise RuntimeError('no stream with <= 4 distance symbols')
    while len(dsyms) < 4:   # pad the simple code to four symbols (2-bit codes)
        extra = [x for x in range(16, 64) if x not in dsyms]
        dsyms = sorted(dsyms + [rng.choice(extra)])
    mlen = pos
    w = Bits()
    w.put(1, 0)           # WBITS 16
    w.put(1, 1)           # ISLAST
    w.put(1, 0)           # ISLASTEMPTY
    nib = max(4, ((mlen - 1).bit_length() + 3) // 4)
    w.put(2, nib - 4)
    w.put(4 * nib, mlen - 1)
    w.put(1, 0)           # NBLTYPESL 1
    w.put(1, 0)           # NBLTYPESI 1
    w.put(1, 0)           # NBLTYPESD 1
    w.put(2, 0)           # NPOSTFIX
    w.put(4, 0)           # NDIRECT
    w.put(2, 0)           # context mode LSB6
    w.put(1, 0)           # NTREESL 1
    w.put(1, 0)           # NTREESD 1
    simple_code(w, 8, [ord('a'), ord('b')])
    simple_code(w, 10, cmds)
    simple_code(w, 6, dsyms)
    w.put(1, 0)           # tree select 0: four 2-bit codes
    for sym, ic, ins, cc, cl, lits, d in prog:
        w.put(1, cmds.index(sym))
        w.put(INS_EXTRA[ic], ins - INS_BASE[ic])
        w.put(COPY_EXTRA[cc], cl - COPY_BASE[cc])
        for c in lits:
            w.put(1, 0 if c == ord('a') else 1)
        ds, nb, extra = dist_symbol(d)
        w.put(2, rev2(dsyms.index(ds)))
        w.put(nb, extra)
    return w.bytes()


def main():
    rng = random.Random(0xD1C7)
    jobs, meta = [], []
    for n in range(160):
        dlen = rng.choice([0, 1, 5, 50, 300, 1000, 4096, 40000])
        dspec = {'kind': 'xorshift', 'seed': 0xD1C70000 + n, 'len': dlen}
        dic = _inputs.resolve(dspec)
        st = make_stream(rng, dlen, good=n % 3 != 2)
        for int8 in (False, True):
            jobs.append({'id': len(jobs), 'op': 'decode', 'variant': 'asis', 'in_b64': base64.b64encode(st).decode(),
                         'dict_b64': base64.b64encode(dic).decode(), 'dict_int8': int8})
            meta.append((st, dspec, int8))
    with tempfile.TemporaryDirectory() as td:
        jf, rf = os.path.join(td, 'j.json'), os.path.join(td, 'r.json')
        with open(jf, 'w') as f:
            json.dump(jobs, f)
        subprocess.run(['node', RUN, jf, rf], check=True)
        with open(rf) as f:
            res = json.load(f)
    cases = []
    for r, (st, dspec, int8) in zip(res, meta):
        c = {'in_b64': base64.b64encode(st).decode(), 'dict': dspec, 'int8': int8}
        if 'error' in r:
            c['error'] = r['error']
        else:
            c['len'] = r['len']
            c['sha256'] = r['sha256']
        cases.append(c)
    ok = sum(1 for c in cases if 'error' not in c)
    with open(OUT, 'w') as f:
        json.dump({'generator': 'oracle/refgen/make_compound.py', 'reference': 'type-erased countertype/brotli-lib '
                   'src/decode (oracle/_ref/asis)', 'cases': cases}, f)
    print('%d cases, %d decoded, %d errors: %s' % (len(cases), ok, len(cases) - ok,
                                                    sorted(set(c['error'] for c in cases if 'error' in c))))


if __name__ == '__main__':
    main()
