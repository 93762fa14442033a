"""DP timing experiment (MIB_PROF build via BROTLI_AMD_LIB): 1024 x 1 MiB text streams
encoded at q11; prints the dp kernel's per-phase cycle counters per segment."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'brotli-lib_amd', 'python'))
import torch  # noqa: E402
import brotli_amd  # noqa: E402
from brotli_amd import datagen  # noqa: E402

k, size = int(os.environ.get('K', '1024')), 1 << 20
dev = torch.device('cuda', 0)
data = datagen.enwik_device(k * size, 7, dev)
ctx = brotli_amd.DeviceContext(0, profiling=True)
cap = k * size + k * 8192
comp = torch.empty(cap, dtype=torch.uint8, device=dev)
lib = brotli_amd._L()
prof = (ctypes.c_ulonglong * 8)()
names = ['stage_cyc', 'node_cyc', 'long_cyc', 'relax_cyc', 'steps', 'chunks', 'stages', 'jumps']
nseg = k * size // 65536
for it in range(2):
    if hasattr(lib, 'mib_debug_read_dp_prof'):
        lib.mib_debug_read_dp_prof(prof)
    off = ctx.encode(data.data_ptr(), [i * size for i in range(k + 1)], comp.data_ptr(), cap, {'quality': 11})
    t = ctx.kernel_times()
    print(it, {n: round(v[0], 2) for n, v in t.items()}, 'ratio', off[-1] / (k * size), flush=True)
    if hasattr(lib, 'mib_debug_read_dp_prof'):
        lib.mib_debug_read_dp_prof(prof)
        d = {n: v / nseg for n, v in zip(names, prof)}
        print({n: round(v, 1) for n, v in d.items()}, flush=True)
        st = max(1.0, d['steps'])
        print('per step: node %.1f relax %.1f stage %.1f long %.1f cycles; chunks/step %.2f' % (
            d['node_cyc'] / st, d['relax_cyc'] / st, d['stage_cyc'] / st, d['long_cyc'] / st, d['chunks'] / st), flush=True)
