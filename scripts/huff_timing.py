"""Huffman-kernel timing experiment (MIB_PROF build via BROTLI_AMD_LIB): per built prefix code,
count-limit attempts and cycles in the rank sort / tree construction / serialisation, on the
C3 and C4 bench batches."""
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
prof = (ctypes.c_ulonglong * 12)()
names = ['trees', 'attempts', 'sort_cyc', 'tree_cyc', 'store_cyc', 'block_cyc', 'symbols', 'retried', 'max_block', 'max_sort', 'max_tree', 'max_store']
ctx = brotli_amd.DeviceContext(0, profiling=True)
if os.environ.get('CADENCE'):   # the reference's cadence: one BrotliEncoder, 1 MiB update() calls
    from brotli_amd import datagen
    text = datagen.enwik_text(16 << 20, 3)
    lib.mib_debug_read_huff_prof(prof)
    enc = brotli_amd.BrotliEncoder({'quality': 9, 'lgwin': 24})
    for i in range(16):
        enc.update(text[i << 20:(i + 1) << 20])
    enc.finish()
    lib.mib_debug_read_huff_prof(prof)
    d = dict(zip(names, list(prof)))
    tr = max(1, d['trees'])
    print('cadence', {n: (v if n.startswith('max') else round(v / tr, 1)) for n, v in d.items() if n != 'trees'}, 'trees', d['trees'],
          flush=True)
    sys.exit(0)
for wl in os.environ.get('WLS', 'c3,c4').split(','):
    k, size, mode, _, _ = bench.WORKLOADS[wl]
    data = bench.make_inputs(wl, k, size, 0, dev)
    cap = k * size + k * size // 8 + 4096 * k
    comp = torch.empty(cap, dtype=torch.uint8, device=dev)
    for it in range(2):
        lib.mib_debug_read_huff_prof(prof)
        off = ctx.encode(data.data_ptr(), [i * size for i in range(k + 1)], comp.data_ptr(), cap, {'quality': 11, 'mode': mode})
        t = ctx.kernel_times()
        lib.mib_debug_read_huff_prof(prof)
        d = dict(zip(names, list(prof)))
        tr = max(1, d['trees'])
        print(wl, it, 'huffman %.2f ms' % t.get('huffman', (0, 0))[0], 'cluster %.2f ms' % t.get('cluster', (0, 0))[0],
              {n: (v if n.startswith('max') else round(v / tr, 1)) for n, v in d.items() if n != 'trees'}, 'trees', d['trees'], flush=True)
