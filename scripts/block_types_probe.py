"""How many block types per category the encoder's split keeps: K streams of C4's
and C3's shapes encoded (BROTLI_AMD_LIB / MIB_* knobs as set by the caller), each decoded by the
oracle, the largest (literal, command, distance) type counts tallied."""
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'brotli-lib_amd', 'python'))
sys.path.insert(0, os.path.join(ROOT, 'tests'))
import _oracle  # noqa: E402
import brotli_amd  # noqa: E402
from brotli_amd import datagen  # noqa: E402

k = int(os.environ.get('K', '48'))
for name, bufs, mode in (('c4', [datagen.enwik_text(1 << 20, 100 + i) for i in range(k)], 0),
                         ('c3', datagen.glyf_font_batch(k, 1 << 18, 1000, workers=8), 2)):
    outs = brotli_amd.encode_batch(bufs, {'quality': 11, 'mode': mode})
    tally = [collections.Counter() for _ in range(3)]
    for b, e in zip(bufs, outs):
        _oracle.max_block_types()
        assert _oracle.decode(e) == b
        for c, v in enumerate(_oracle.max_block_types()):
            tally[c][v] += 1
    ratio = sum(map(len, outs)) / sum(map(len, bufs))
    print(name, 'ratio %.5f' % ratio, 'literal', dict(sorted(tally[0].items())), 'command', dict(sorted(tally[1].items())),
          'distance', dict(sorted(tally[2].items())), flush=True)
