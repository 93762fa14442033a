"""Part-parallel decode diagnostics: which bytes differ, against which part boundaries."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'brotli-lib_amd', 'python'))
sys.path.insert(0, os.path.join(ROOT, 'tests'))
import brotli_amd  # noqa: E402
import _parts  # noqa: E402
from brotli_amd import datagen  # noqa: E402


def report(name, data, enc):
    ents, total = _parts.read_chain(enc)
    p0, f0 = brotli_amd.part_stats()
    got = brotli_amd.brotliDecode(enc)
    p1, f1 = brotli_amd.part_stats()
    a = np.frombuffer(data, np.uint8)
    b = np.frombuffer(got, np.uint8)
    ok = len(a) == len(b) and np.array_equal(a, b)
    print(name, 'parts', len(ents), 'parallel', p1 - p0, 'fallback', f1 - f0, 'ok', ok, flush=True)
    if not ok and len(a) == len(b):
        d = np.nonzero(a != b)[0]
        print('  ndiff', len(d), flush=True)
        pos = ents['pos'].astype(np.int64)
        runs = []
        s = d[0]
        prev = d[0]
        for x in d[1:]:
            if x != prev + 1:
                runs.append((s, prev + 1))
                s = x
            prev = x
        runs.append((s, prev + 1))
        for r0, r1 in runs[:40]:
            k = int(np.searchsorted(pos, r0, side='right')) - 1
            print('  diff [%d, %d) len %d in part %d (starts %d, +%d)' % (r0, r1, r1 - r0, k, pos[k], r0 - pos[k]), flush=True)


data = datagen.enwik_text(20 << 20, 9)
for q, lg in ((9, 24), (11, 24), (9, 22)):
    enc = brotli_amd.brotliEncode(data, {'quality': q, 'lgwin': lg})
    report('oneshot q%d lgwin%d' % (q, lg), data, enc)
e = brotli_amd.BrotliEncoder({'quality': 9, 'lgwin': 24})
parts = [e.update(data[i:i + (1 << 20)]) for i in range(0, len(data), 1 << 20)]
parts.append(e.finish())
report('streaming q9 lgwin24', data, b''.join(parts))
e = brotli_amd.BrotliEncoder({'quality': 9, 'lgwin': 22})
parts = [e.update(data[i:i + (1 << 20)]) for i in range(0, len(data), 1 << 20)]
parts.append(e.finish())
report('streaming q9 lgwin22', data, b''.join(parts))
