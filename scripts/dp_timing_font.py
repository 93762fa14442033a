"""DP timing experiment (MIB_PROF build via BROTLI_AMD_LIB) on C3's shape: K x 256 KiB
WOFF2-transformed glyf buffers at q11 FONT; the dp kernel's per-phase cycle counters per
segment (slot 5: the distance-cache candidates' cycles)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'brotli-lib_amd', 'python'))
import torch  # noqa: E402
import brotli_amd  # noqa: E402
from brotli_amd import datagen  # noqa: E402

k, size = int(os.environ.get('K', '256')), 1 << 18
bufs = datagen.glyf_font_batch(k, size, 1000, workers=8)
dev = torch.device('cuda', 0)
data = torch.frombuffer(bytearray(b''.join(bufs)), dtype=torch.uint8).to(dev)
ctx = brotli_amd.DeviceContext(0, profiling=True)
cap = k * size + k * 8192
comp = torch.empty(cap, dtype=torch.uint8, device=dev)
lib = brotli_amd._L()
prof = (ctypes.c_ulonglong * 8)()
names = ['stage_cyc', 'node_cyc', 'long_cyc', 'relax_cyc', 'steps', 'kc_cyc', 'kc1_cyc', 'kc_iters']
nseg = k * size // 65536
lib.mib_force_no_dp_cache.argtypes = [ctypes.c_int]
for it in range(4):
    lib.mib_force_no_dp_cache(1 if it >= 2 else 0)   # (the last two: without the candidates)
    lib.mib_debug_read_dp_prof(prof)
    off = ctx.encode(data.data_ptr(), [i * size for i in range(k + 1)], comp.data_ptr(), cap, {'quality': 11, 'mode': 2})
    t = ctx.kernel_times()
    print(it, {n: round(v[0], 2) for n, v in t.items() if v[0] > 0.5}, 'ratio', off[-1] / (k * size), flush=True)
    lib.mib_debug_read_dp_prof(prof)
    d = {n: v / nseg for n, v in zip(names, prof)}
    st = max(1.0, d['steps'])
    print('per step: node %.1f relax %.1f kc measure+relax %.1f kc ring+issue %.1f stage %.1f long %.1f cycles' % (
        d['node_cyc'] / st, d['relax_cyc'] / st, d['kc1_cyc'] / st, d['kc_cyc'] / st, d['stage_cyc'] / st, d['long_cyc'] / st), flush=True)
    print('candidate loop: iterations per step %.3f (the long-copy slot counts steps with a passing candidate: %.3f)' % (
        d['kc_iters'] / st, d['long_cyc'] / st), flush=True)
