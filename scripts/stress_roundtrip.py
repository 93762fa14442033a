"""Randomised round trips: sizes, qualities, windows, modes and generators, encoded on the GPU,
decoded by the oracle (the reference decoder restated) and by the HIP decoder."""
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'brotli-lib_amd', 'python'))
sys.path.insert(0, os.path.join(ROOT, 'tests'))
import _oracle  # noqa: E402
import brotli_amd  # noqa: E402
from brotli_amd import datagen  # noqa: E402

rng = random.Random(int(sys.argv[1]) if len(sys.argv) > 1 else 1)
t0 = time.time()
n_ok = 0
while time.time() - t0 < float(sys.argv[2]) if len(sys.argv) > 2 else 60:
    kind = rng.choice(['text', 'glyf', 'random', 'mixed', 'runs', 'records', 'records', 'records_text'])
    n = rng.choice([rng.randint(0, 300), rng.randint(300, 70000), rng.randint(70000, 600000), rng.randint(2 << 20, 3 << 20)])
    seed = rng.randint(0, 10 ** 6)
    if kind == 'text':
        d = datagen.enwik_text(n, seed)
    elif kind == 'glyf':
        d = datagen.glyf_stream(n, seed)
    elif kind == 'random':
        d = bytes(rng.getrandbits(8) for _ in range(min(n, 200000)))
    elif kind in ('records', 'records_text'):
        # binary records repeating one to four records back with bytes changed (the parse's
        # distance-cache candidates run on such data: non-UTF-8 literals)
        rec = rng.randint(8, 300)
        out = bytearray(rng.getrandbits(8) for _ in range(rec * 4))
        while len(out) < n:
            back = rec * rng.randint(1, 4) + (rng.randint(-3, 3) if rng.random() < 0.1 else 0)
            back = max(1, min(back, len(out)))
            r = bytearray(out[len(out) - back:len(out) - back + rec])
            for _ in range(rng.randint(0, 4)):
                r[rng.randrange(len(r))] = rng.getrandbits(8)
            out += r
        d = bytes(out[:n])
        if kind == 'records_text':
            d = datagen.enwik_text(n // 3, seed) + d[:n - n // 3]
    elif kind == 'runs':
        d = b''.join(bytes([rng.randint(0, 3)]) * rng.randint(1, 300) for _ in range(max(1, n // 150)))[:n]
    else:
        d = datagen.enwik_text(n // 2, seed) + datagen.glyf_stream(n - n // 2, seed)
    q = rng.choice([5, 9, 10, 11, 11, 11])
    lg = rng.choice([16, 18, 22, 22, 24])
    mode = rng.choice([0, 1, 2])
    enc = brotli_amd.brotliEncode(d, {'quality': q, 'lgwin': lg, 'mode': mode})
    if _oracle.decode(enc) != d or brotli_amd.brotliDecode(enc) != d:
        print('FAIL', kind, len(d), seed, q, lg, mode, flush=True)
        sys.exit(1)
    n_ok += 1
    if n_ok % 100 == 0:
        print(n_ok, 'round trips', round(time.time() - t0), 's', flush=True)
print('ok', n_ok, 'round trips', flush=True)
