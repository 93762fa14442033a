"""C1 latency diagnostics: one 45,000 B enwik-style text, brotliEncode (q11) then brotliDecode
through the host API; per call: wall time and the decoder's kernel time / launches (HIP
events, default_profiling), and the stream's shape from the oracle's decoder."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'brotli-lib_amd', 'python'))
import brotli_amd  # noqa: E402
from brotli_amd import datagen  # noqa: E402

data = datagen.enwik_text(45000, 1)
enc = brotli_amd.brotliEncode(data, {'quality': 11})
print('stream', len(enc), 'bytes', flush=True)
for _ in range(3):
    assert brotli_amd.brotliDecode(enc) == data
brotli_amd.default_profiling(True)
for it in range(5):
    brotli_amd.default_profiling(True)
    t0 = time.perf_counter()
    out = brotli_amd.brotliDecode(enc)
    t1 = time.perf_counter()
    print('decode wall %.3f ms' % ((t1 - t0) * 1e3), brotli_amd.default_kernel_times(), flush=True)
with open(os.path.join(ROOT, 'gpurun_out', 'c1_stream.br'), 'wb') as f:
    f.write(enc)
