"""Block-split timing experiment (MIB_PROF build via BROTLI_AMD_LIB): thread 0's cycles per
phase of split_kernel (load, seed, type histograms, costs, unit costs, shortest path, final
cost, serial tail), per (metablock, category) block, on the C2 and C4 bench batches."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'brotli-lib_amd', 'python'))
import torch  # noqa: E402
import brotli_amd  # noqa: E402
import bench  # noqa: E402

dev = torch.device('cuda', 0)
lib = brotli_amd._L()
prof = (ctypes.c_ulonglong * 8)()
names = ['load', 'seed', 'histo', 'costs', 'unit_costs', 'path', 'final', 'tail']
ctx = brotli_amd.DeviceContext(0, profiling=True)
if os.environ.get('CADENCE'):   # the reference's cadence: one BrotliEncoder, 1 MiB update() calls
    from brotli_amd import datagen
    text = datagen.enwik_text(16 << 20, 3)
    lib.mib_debug_read_split_prof(prof)
    enc = brotli_amd.BrotliEncoder({'quality': 9, 'lgwin': 24})
    for i in range(16):
        enc.update(text[i << 20:(i + 1) << 20])
    enc.finish()
    lib.mib_debug_read_split_prof(prof)
    nblk = 3 * 17   # (metablocks: 16 chunks + the final one; three categories)
    print('cadence', {n: round(v / nblk) for n, v in zip(names, list(prof))}, flush=True)
    sys.exit(0)
for wl in os.environ.get('WLS', 'c2,c4').split(','):
    k, size, mode, _, _ = bench.WORKLOADS[wl]
    data = bench.make_inputs(wl, k, size, 0, dev)
    cap = k * size + k * size // 8 + 4096 * k
    comp = torch.empty(cap, dtype=torch.uint8, device=dev)
    nblk = 3 * ((size + (16 << 20) - 1) // (16 << 20)) * k
    for it in range(2):
        lib.mib_debug_read_split_prof(prof)
        ctx.encode(data.data_ptr(), [i * size for i in range(k + 1)], comp.data_ptr(), cap, {'quality': 11, 'mode': mode})
        t = ctx.kernel_times()
        lib.mib_debug_read_split_prof(prof)
        print(wl, it, 'block_split %.2f ms' % t.get('block_split', (0, 0))[0],
              {n: round(v / nblk) for n, v in zip(names, list(prof))}, flush=True)
