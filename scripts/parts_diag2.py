import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'brotli-lib_amd', 'python'))
sys.path.insert(0, os.path.join(ROOT, 'tests'))
import brotli_amd  # noqa: E402
import _parts  # noqa: E402
from brotli_amd import datagen  # noqa: E402

data = datagen.enwik_text(20 << 20, 9)
a = np.frombuffer(data, np.uint8)
for lg, q, chunkmb in ((24, 9, 1), (23, 9, 1), (24, 11, 1), (24, 9, 4)):
    e = brotli_amd.BrotliEncoder({'quality': q, 'lgwin': lg})
    step = chunkmb << 20
    parts = [e.update(data[i:i + step]) for i in range(0, len(data), step)]
    parts.append(e.finish())
    enc = b''.join(parts)
    ents, total = _parts.read_chain(enc)
    for rep in range(3):
        got = brotli_amd.brotliDecode(enc)
        b = np.frombuffer(got, np.uint8)
        d = np.nonzero(a != b)[0] if len(a) == len(b) else None
        print('lg', lg, 'q', q, 'rep', rep, 'len ok', len(a) == len(b), 'ndiff', None if d is None else len(d),
              'first', None if d is None or len(d) == 0 else (int(d[0]), bytes(b[d[0]:d[0] + 8]), bytes(a[d[0]:d[0] + 8])), flush=True)
    print('  chunk heads at', [i for i in range(len(enc)) if False], 'npos', len(ents), 'first entries', ents['pos'][:3], ents['bit'][:3], flush=True)
    # where is the stream's byte 1..4 data referenced?  print the index positions near chunk starts
    cs = [int(x) for x in ents['pos'] if int(x) % (8 << 20) == 0]
    print('  chunk-start entries', cs, flush=True)
