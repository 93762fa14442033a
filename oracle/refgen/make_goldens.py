#!/usr/bin/env python3
"""Generate tests/golden/*.json by running the type-erased reference itself
(oracle/_ref, built by erase_ts.py) on Node 12 in this container.

TEST INFRASTRUCTURE ONLY.  The fixtures are data (inputs as specs, expected outputs as
bytes/hashes); the reference never leaves this container.

  encode_ref_fixed.json  brotliEncode outputs of the A+B-fixed reference ("ref-fixed"),
                         plus the as-is reference's sizes where they differ
  decode_errors.json     brotliDecode on corrupted / truncated / random streams (as-is
                         reference): output hash or "Brotli error code: N"
  decode_vectors.json    sha256/len of the reference decoder's output on every .br we ship
  bt_matches.json        per-position binary-tree match lists (ref-fixed), pinning a2/a3

usage: python3 oracle/refgen/make_goldens.py [--only encode,decode,bt]
"""
import argparse
import base64
import concurrent.futures as cf
import glob
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
GOLD = os.path.join(ROOT, 'tests', 'golden')


def run_jobs(jobs, tmp):
    jf = os.path.join(tmp, 'jobs_%d.json' % id(jobs))
    rf = jf + '.out'
    with open(jf, 'w') as f:
        json.dump(jobs, f)
    subprocess.run(['node', RUN, jf, rf], check=True, stderr=subprocess.DEVNULL)
    with open(rf) as f:
        return json.load(f)


def encode_cases():
    cases = []
    # the reference's fuzz corpus (test/brotli.test.ts:263-281), one generator across sizes
    seed = 0xC0FFEE ^ 0xBEEF
    skip = 0
    for size in [0, 1, 2, 3, 4, 7, 15, 31, 63, 64, 65, 127, 255, 256, 257, 511, 1024, 2048]:
        for spec in ({'kind': 'xorshift', 'seed': seed, 'skip': skip, 'len': size}, {'kind': 'ramp', 'len': size}):
            for q in (0, 10, 11):
                cases.append((spec, {'quality': q}))
        skip += size
    texts = [
        {'kind': 'text', 's': 'Hello, World!'},
        {'kind': 'text', 's': 'Test quality 11 encoding'},
        {'kind': 'fox', 'repeats': 100},
        {'kind': 'fox', 'repeats': 1000},
        {'kind': 'file', 'path': 'vectors/alice29.txt', 'len': 1000},
        {'kind': 'file', 'path': 'vectors/alice29.txt', 'len': 4096},
        {'kind': 'file', 'path': 'vectors/alice29.txt', 'len': 45000},
        {'kind': 'file', 'path': 'vectors/asyoulik.txt', 'len': 20000},
        {'kind': 'file', 'path': 'vectors/plrabn12.txt', 'off': 10000, 'len': 45000},
        {'kind': 'file', 'path': 'vectors/lcet10.txt', 'len': 120000},
        {'kind': 'enwik', 'seed': 1, 'len': 45000},
        {'kind': 'enwik', 'seed': 2, 'len': 200000},
        {'kind': 'file', 'path': 'bench/html-content.bin'},
        {'kind': 'file', 'path': 'bench/random-binary.bin'},
        {'kind': 'file', 'path': 'vectors/zeros'},
        {'kind': 'file', 'path': 'vectors/zerosukkanooa'},
        {'kind': 'file', 'path': 'vectors/backward65536'},
        {'kind': 'file', 'path': 'vectors/quickfox_repeated'},
        {'kind': 'file', 'path': 'vectors/compressed_repeated'},
        {'kind': 'file', 'path': 'vectors/cp1251-utf16le'},
        {'kind': 'file', 'path': 'vectors/cp852-utf8'},
        {'kind': 'file', 'path': 'vectors/monkey'},
        {'kind': 'file', 'path': 'vectors/ukkonooa'},
        {'kind': 'file', 'path': 'vectors/random_chunks'},
        {'kind': 'file', 'path': 'vectors/mapsdatazrh'},
    ]
    for spec in texts:
        cases.append((spec, {'quality': 11}))
    for spec in texts[4:8] + texts[10:11]:
        cases.append((spec, {'quality': 10}))
    fonts = [
        {'kind': 'file', 'path': 'bench/enc-ttf.bin', 'len': 4096},
        {'kind': 'file', 'path': 'bench/enc-ttf.bin', 'len': 65536},
        {'kind': 'file', 'path': 'bench/enc-ttf.bin', 'len': 262144},
        {'kind': 'file', 'path': 'bench/enc-otf.bin', 'len': 100000},
        {'kind': 'glyf', 'seed': 1000, 'len': 65536},
    ]
    for spec in fonts:
        cases.append((spec, {'quality': 11, 'mode': 2}))
    cases.append((fonts[1], {'quality': 11}))
    # window sizes (inputs kept below 2^lgwin - 16: larger ones hit bugs C/E in the reference)
    for lg, spec in ((10, {'kind': 'file', 'path': 'vectors/alice29.txt', 'len': 900}),
                     (16, {'kind': 'file', 'path': 'vectors/alice29.txt', 'len': 45000}),
                     (18, {'kind': 'file', 'path': 'vectors/alice29.txt', 'len': 45000}),
                     (24, {'kind': 'file', 'path': 'vectors/alice29.txt', 'len': 45000})):
        cases.append((spec, {'quality': 11, 'lgwin': lg}))
    return cases


def gen_encode(tmp):
    cases = encode_cases()
    jobs = []
    for i, (spec, opts) in enumerate(cases):
        data = _inputs.resolve(spec)
        p = os.path.join(tmp, 'in_%d' % i)
        with open(p, 'wb') as f:
            f.write(data)
        for variant in ('fixed', 'asis'):
            jobs.append({'id': '%d_%s' % (i, variant), 'op': 'encode', 'variant': variant, 'in': p, 'opts': opts,
                         'inline_max': 6000 if variant == 'fixed' else 0})
    # spread over 8 processes
    chunks = [jobs[k::8] for k in range(8)]
    res = {}
    with cf.ThreadPoolExecutor(8) as ex:
        for out in ex.map(lambda c: run_jobs(c, tmp), chunks):
            for r in out:
                res[r['id']] = r
    golden = []
    for i, (spec, opts) in enumerate(cases):
        fx, asis = res['%d_fixed' % i], res['%d_asis' % i]
        g = {'input': spec, 'opts': opts, 'len': fx['len'], 'sha256': fx['sha256'], 'ref_ms': round(fx['ms'], 3),
             'native_roundtrip': fx['native_roundtrip']}
        if 'out_b64' in fx:
            g['out_b64'] = fx['out_b64']
        if asis.get('sha256') != fx['sha256']:
            g['asis_len'] = asis.get('len')
            g['asis_sha256'] = asis.get('sha256')
            g['asis_native_roundtrip'] = asis.get('native_roundtrip')
        golden.append(g)
    with open(os.path.join(GOLD, 'encode_ref_fixed.json'), 'w') as f:
        json.dump({'generator': 'oracle/refgen/make_goldens.py', 'reference': 'countertype/brotli-lib v0.0.7, A+B fixed',
                   'cases': golden}, f, indent=0)
    print('encode goldens:', len(golden))


def decode_one(args):
    tmp, i, blob, opts = args
    jf = os.path.join(tmp, 'd_%d.json' % i)
    job = [{'id': str(i), 'op': 'decode', 'variant': 'asis', 'in_b64': base64.b64encode(blob).decode()}]
    if opts is not None:
        job[0]['opts'] = opts
    with open(jf, 'w') as f:
        json.dump(job, f)
    try:
        subprocess.run(['node', RUN, jf, jf + '.out'], check=True, stderr=subprocess.DEVNULL, timeout=20)
    except subprocess.TimeoutExpired:
        return {'id': str(i), 'hang': True}
    with open(jf + '.out') as f:
        return json.load(f)[0]


def gen_decode(tmp):
    rng = random.Random(0xB207)
    sources = []
    for f in sorted(glob.glob(os.path.join(GOLD, 'vectors', '*.compressed*'))):
        b = open(f, 'rb').read()
        if len(b) <= 2048:
            sources.append(b)
    # two encoder outputs with context maps / block splits (ref-fixed q11)
    for spec, opts in (({'kind': 'file', 'path': 'vectors/alice29.txt', 'len': 3000}, {'quality': 11}),
                       ({'kind': 'file', 'path': 'bench/enc-ttf.bin', 'len': 3000}, {'quality': 11, 'mode': 2})):
        p = os.path.join(tmp, 'src_%d' % len(sources))
        with open(p, 'wb') as f:
            f.write(_inputs.resolve(spec))
        r = run_jobs([{'id': 'x', 'op': 'encode', 'variant': 'fixed', 'in': p, 'opts': opts, 'inline_max': 1 << 20}], tmp)[0]
        sources.append(base64.b64decode(r['out_b64']))
    blobs = []
    for s in sources:
        cuts = range(len(s)) if len(s) <= 48 else sorted(rng.sample(range(len(s)), 24))
        for c in cuts:
            blobs.append(s[:c])
        for _ in range(12 if len(s) > 16 else 4):
            bb = bytearray(s)
            k = rng.randrange(len(bb) * 8)
            bb[k >> 3] ^= 1 << (k & 7)
            blobs.append(bytes(bb))
        for extra in (b'\x00', b'\xff', b'\x01\x02\x03'):
            blobs.append(s + extra)
    for _ in range(60):
        blobs.append(bytes(rng.randrange(256) for _ in range(rng.randrange(1, 64))))
    # dedupe, keep order
    seen, uniq = set(), []
    for b in blobs:
        if b not in seen:
            seen.add(b)
            uniq.append(b)
    args = [(tmp, i, b, None) for i, b in enumerate(uniq)]
    with cf.ThreadPoolExecutor(8) as ex:
        res = list(ex.map(decode_one, args))
    cases = []
    for b, r in zip(uniq, res):
        c = {'in_b64': base64.b64encode(b).decode()}
        if r.get('hang'):
            c['hang'] = True
        elif 'error' in r:
            c['error'] = r['error']
        else:
            c['len'] = r['len']
            c['sha256'] = r['sha256']
        cases.append(c)
    with open(os.path.join(GOLD, 'decode_errors.json'), 'w') as f:
        json.dump({'generator': 'oracle/refgen/make_goldens.py', 'reference': 'countertype/brotli-lib v0.0.7 (as is)',
                   'cases': cases}, f, indent=0)
    nerr = sum('error' in c for c in cases)
    print('decode goldens:', len(cases), 'errors', nerr)
    # full decode of every shipped .br / .compressed stream
    vec = []
    for f in sorted(glob.glob(os.path.join(GOLD, 'vectors', '*.compressed*')) + glob.glob(os.path.join(GOLD, 'bench', '*.br'))):
        r = run_jobs([{'id': 'v', 'op': 'decode', 'variant': 'asis', 'in': f}], tmp)[0]
        vec.append({'path': os.path.relpath(f, GOLD), 'len': r.get('len'), 'sha256': r.get('sha256'), 'error': r.get('error')})
    with open(os.path.join(GOLD, 'decode_vectors.json'), 'w') as f:
        json.dump({'generator': 'oracle/refgen/make_goldens.py', 'cases': vec}, f, indent=0)
    print('decode vectors:', len(vec))


def q59_cases():
    """brotliEncode at qualities 5-9 (hash chains + greedy, backward-references.ts:14-134): one-shot
    inputs below 2^lgwin (past it the reference's ring indexing is wrong: bugs C/E), lgwin 22 and
    others, GENERIC / TEXT / FONT."""
    ins = [
        {'kind': 'file', 'path': 'vectors/alice29.txt', 'len': 45000},
        {'kind': 'file', 'path': 'vectors/asyoulik.txt', 'len': 20000},
        {'kind': 'file', 'path': 'vectors/lcet10.txt', 'len': 120000},
        {'kind': 'enwik', 'seed': 1, 'len': 45000},
        {'kind': 'enwik', 'seed': 3, 'len': 300000},
        {'kind': 'fox', 'repeats': 1000},
        {'kind': 'file', 'path': 'bench/html-content.bin'},
        {'kind': 'file', 'path': 'bench/random-binary.bin'},
        {'kind': 'file', 'path': 'vectors/zerosukkanooa'},
        {'kind': 'file', 'path': 'vectors/quickfox_repeated'},
        {'kind': 'file', 'path': 'vectors/mapsdatazrh'},
        {'kind': 'file', 'path': 'vectors/random_chunks'},
        {'kind': 'xorshift', 'seed': 77, 'skip': 0, 'len': 200},
        {'kind': 'ramp', 'len': 3000},
    ]
    cases = []
    for q in (5, 6, 7, 8, 9):
        for spec in ins:
            cases.append((spec, {'quality': q}))
    for q in (5, 7, 9):
        cases.append(({'kind': 'file', 'path': 'bench/enc-ttf.bin', 'len': 262144}, {'quality': q, 'mode': 2}))
        cases.append(({'kind': 'glyf', 'seed': 1001, 'len': 65536}, {'quality': q, 'mode': 2}))
        cases.append(({'kind': 'file', 'path': 'vectors/alice29.txt', 'len': 45000}, {'quality': q, 'mode': 1}))
        cases.append(({'kind': 'file', 'path': 'vectors/alice29.txt', 'len': 30000}, {'quality': q, 'lgwin': 16}))
        cases.append(({'kind': 'enwik', 'seed': 4, 'len': 1 << 20}, {'quality': q, 'lgwin': 24}))
    cases.append(({'kind': 'enwik', 'seed': 5, 'len': (4 << 20) - 64}, {'quality': 9, 'lgwin': 22}))
    return cases


def gen_q59(tmp):
    cases = q59_cases()
    jobs = []
    for i, (spec, opts) in enumerate(cases):
        p = os.path.join(tmp, 'q_%d' % i)
        with open(p, 'wb') as f:
            f.write(_inputs.resolve(spec))
        jobs.append({'id': str(i), 'op': 'encode', 'variant': 'fixed', 'in': p, 'opts': opts, 'inline_max': 0})
    chunks = [jobs[k::8] for k in range(8)]
    res = {}
    with cf.ThreadPoolExecutor(8) as ex:
        for out in ex.map(lambda c: run_jobs(c, tmp), chunks):
            for r in out:
                res[r['id']] = r
    golden = []
    for i, (spec, opts) in enumerate(cases):
        r = res[str(i)]
        golden.append({'input': spec, 'opts': opts, 'len': r['len'], 'sha256': r['sha256'], 'ref_ms': round(r['ms'], 3),
                       'native_roundtrip': r['native_roundtrip']})
    with open(os.path.join(GOLD, 'encode_ref_q5_9.json'), 'w') as f:
        json.dump({'generator': 'oracle/refgen/make_goldens.py --only q59',
                   'reference': 'countertype/brotli-lib v0.0.7 (the q5-9 path: hash chains + greedy, as is)',
                   'cases': golden}, f, indent=0)
    print('q5-9 encode goldens:', len(golden))


def gen_bt(tmp):
    out = []
    for spec in ({'kind': 'file', 'path': 'vectors/alice29.txt', 'len': 4096},
                 {'kind': 'file', 'path': 'bench/enc-ttf.bin', 'len': 4096},
                 {'kind': 'file', 'path': 'vectors/zerosukkanooa', 'len': 4096}):
        p = os.path.join(tmp, 'bt_in')
        with open(p, 'wb') as f:
            f.write(_inputs.resolve(spec))
        r = run_jobs([{'id': 'b', 'op': 'bt_matches', 'variant': 'fixed', 'in': p}], tmp)[0]
        out.append({'input': spec, 'lists': r['lists']})
    with open(os.path.join(GOLD, 'bt_matches.json'), 'w') as f:
        json.dump({'generator': 'oracle/refgen/make_goldens.py', 'cases': out}, f)
    print('bt goldens:', len(out))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--only', default='encode,decode,bt')
    a = ap.parse_args()
    with tempfile.TemporaryDirectory() as tmp:
        for part in a.only.split(','):
            {'encode': gen_encode, 'decode': gen_decode, 'bt': gen_bt, 'q59': gen_q59}[part](tmp)


if __name__ == '__main__':
    main()
