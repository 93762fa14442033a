"""C2 part-decode diagnostics (MIB_PROF build, BROTLI_AMD_LIB): encode the 64 MiB C2 buffer,
decode it part-parallel and print per-part clocks from decode_parts_kernel: start, header
done, end, cycles waiting on earlier parts."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'brotli-lib_amd', 'python'))
import numpy as np  # noqa: E402
import brotli_amd  # noqa: E402
from brotli_amd import datagen  # noqa: E402

lib = brotli_amd._L()
NAMES = ['cmd_tail', 'lit_tail', 'distance', 'copy_rest', 'n_literals', 'n_commands', 'mb_lds_tables', 'mb_hbm_tables',
         'F_cmd', 'F_lit', 'F_dist', 'F_copy', 'F_top', 'copy_readlane', 'fast_cmds', 'fast_calls']
prof = (ctypes.c_ulonglong * 16)()


def counters(div):
    lib.mib_debug_read_prof(prof)
    return {n: round(v / div, 1) for n, v in zip(NAMES, prof)}


# the same occupancy with whole streams: 256 x 1 MiB (one wave per CU, the BIG build)
import torch  # noqa: E402
dev = torch.device('cuda', 0)
ctx = brotli_amd.DeviceContext(0, profiling=True)
k, size = 256, 1 << 20
data = datagen.enwik_device(k * size, 2000, dev)
cap = k * size + k * 8192
comp = torch.empty(cap, dtype=torch.uint8, device=dev)
off = ctx.encode(data.data_ptr(), [i * size for i in range(k + 1)], comp.data_ptr(), cap, {'quality': 11})
slot = size + 4096
dec = torch.empty(k * slot, dtype=torch.uint8, device=dev)
counters(1)
for it in range(int(os.environ.get("C4_ITERS", "2"))):
    ctx.decode(comp.data_ptr(), off, dec.data_ptr(), [i * slot for i in range(k + 1)])
    ok = torch.equal(dec.view(k, slot)[:, :size], data.view(k, size))
    print('256x1MiB', it, ctx.kernel_times(), 'ok' if ok else 'MISMATCH', counters(k), flush=True)
del comp, dec, data
n = int(sys.argv[1]) if len(sys.argv) > 1 else 64 << 20
d = datagen.enwik_text(n, 2)
enc = brotli_amd.brotliEncode(d, {'quality': 11, 'lgwin': 22})
print('compressed', len(enc), len(enc) / n, flush=True)
for it in range(3):
    out = brotli_amd.brotliDecode(enc)
    assert out == d
    print('counters per part', counters(n >> 18), flush=True)
    hp = (ctypes.c_ulonglong * 16)()
    lib.mib_debug_read_hdr_prof(hp)
    hn = ['parts_modes', 'ctx_maps', 'lit_group', 'cmd_group', 'dist_group', 'headers', 'lit_trees', 'code_lengths',
          'build_table', 'lds_copy_rest']
    print('header cycles per header', {k: round(hp[i] / max(1, hp[5]), 1) for i, k in enumerate(hn)}, flush=True)
    buf = (ctypes.c_ulonglong * (8 * 8192))()
    lib.mib_debug_read_part_prof(buf, 8192)
    a = np.frombuffer(buf, dtype=np.uint64).reshape(8192, 8).astype(np.int64)
    k = int((a[:, 1] > 0).sum())
    a = a[:k]
    t0 = a[:, 0].min()
    start, end, hdr = a[:, 0] - t0, a[:, 1] - t0, a[:, 5] - a[:, 0]
    dur = a[:, 1] - a[:, 0]
    mhz = 2400.0   # s_memtime counts shader clocks (~2,400 MHz)
    print('iter', it, 'parts', k, 'span ms %.2f' % ((end.max()) / mhz / 1e3),
          'start ms max %.3f' % (start.max() / mhz / 1e3),
          'dur ms min/med/mean/max %.2f %.2f %.2f %.2f' % tuple(x / mhz / 1e3 for x in (dur.min(), np.median(dur), dur.mean(), dur.max())),
          'hdr ms mean/max %.3f %.3f' % (hdr.mean() / mhz / 1e3, hdr.max() / mhz / 1e3),
          'wait ms mean/max %.3f %.3f' % (a[:, 2].mean() / mhz / 1e3, a[:, 2].max() / mhz / 1e3),
          'waits mean/max %.1f %d spins %d' % (a[:, 3].mean(), a[:, 3].max(), a[:, 4].sum()), flush=True)
    if it == 2:
        order = np.argsort(-dur)
        print('slowest parts (idx, dur ms, wait ms, waits, hwid):')
        for i in order[:12]:
            print('  %d %.2f %.3f %d %x' % (i, dur[i] / mhz / 1e3, a[i, 2] / mhz / 1e3, a[i, 3], a[i, 7]))
        xcc = a[:, 6] & 0xF
        print('xcc of parts 0..63:', ''.join('%x' % x for x in xcc[:64]), ' blocks:', list(a[:16, 6] >> 8))
        same = np.mean(xcc[1:] == xcc[:-1])
        print('parts on the XCD of the part before: %.3f' % same)
        print('dur ms deciles', ['%.1f' % (x / mhz / 1e3) for x in np.percentile(dur, range(0, 101, 10))])
        xcd = (a[:, 7] >> 0)  # raw hw id
        np.save(os.path.join(ROOT, 'gpurun_out', 'c2_part_prof.npy'), a)

# the same stream decoded by one wave (the index's magic spoiled: plan_parts refuses it)
if os.environ.get('SKIP_SERIAL'):
    sys.exit(0)
i = enc.find(b'MBp1')
bad = enc[:i] + b'XBp1' + enc[i + 4:]
import time  # noqa: E402
t = time.time()
out = brotli_amd.brotliDecode(bad)
print('serial', 'ok' if out == d else 'MISMATCH', '%.2f s' % (time.time() - t), counters(n >> 18), flush=True)
