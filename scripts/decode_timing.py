"""Decoder timing experiment: 1024 x 1 MiB text streams encoded on the GPU, then decoded
with kernel timing (correctness not checked: used with instrumented builds)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'brotli-lib_amd', 'python'))
import torch  # noqa: E402
import brotli_amd  # noqa: E402
from brotli_amd import datagen  # noqa: E402

k, size = 1024, 1 << 20
dev = torch.device('cuda', 0)
data = datagen.enwik_device(k * size, 7, dev)
ctx = brotli_amd.DeviceContext(0, profiling=True)
cap = k * size + k * 8192
comp = torch.empty(cap, dtype=torch.uint8, device=dev)
off = ctx.encode(data.data_ptr(), [i * size for i in range(k + 1)], comp.data_ptr(), cap, {'quality': 11})
slot = size + 4096
dec = torch.empty(k * slot, dtype=torch.uint8, device=dev)
import ctypes  # noqa: E402
lib = brotli_amd._L()
prof = (ctypes.c_ulonglong * 16)()
has_prof = hasattr(lib, 'mib_debug_read_prof')
for it in range(3):
    sizes, st = ctx.decode(comp.data_ptr(), off, dec.data_ptr(), [i * slot for i in range(k + 1)])
    print(it, ctx.kernel_times(), 'ok' if torch.equal(dec.view(k, slot)[:, :size], data.view(k, size)) else 'MISMATCH',
          flush=True)
    if has_prof:
        lib.mib_debug_read_prof(prof)
        names = ['cmd_tail', 'lit_tail', 'distance', 'copy_rest', 'n_literals', 'n_commands', 'mb_lds_tables', 'mb_hbm_tables', 'F_cmd', 'F_lit', 'F_dist', 'F_copy', 'F_top', 'copy_readlane', 'fast_cmds', 'fast_calls']
        print({n: v / k for n, v in zip(names, prof)}, flush=True)
