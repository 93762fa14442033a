"""Decoder diagnostics (instrumented MIB_PROF build, BROTLI_AMD_LIB): per-phase cycle counters
of the wave-per-stream decoder on (a) the C4 batch, 1024 x 1 MiB GPU-encoded enwik-style
streams, and (b) each reference bench stream decoded alone; also dumps 16 of the C4 streams
(and their inputs) to gpurun_out/c4_sample/ for CPU-side analysis with the oracle."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'brotli-lib_amd', 'python'))
import torch  # noqa: E402
import brotli_amd  # noqa: E402
from brotli_amd import datagen  # noqa: E402

NAMES = ['cmd_tail', 'lit_tail', 'distance', 'copy_rest', 'n_literals', 'n_commands', 'mb_lds_tables', 'mb_hbm_tables',
         'F_cmd', 'F_lit', 'F_dist', 'F_copy', 'F_top', 'copy_readlane', 'fast_cmds', 'fast_calls']
lib = brotli_amd._L()
prof = (ctypes.c_ulonglong * 16)()
has_prof = hasattr(lib, 'mib_debug_read_prof')


def counters(div):
    if not has_prof:
        return None
    lib.mib_debug_read_prof(prof)
    return {n: round(v / div, 1) for n, v in zip(NAMES, prof)}


dev = torch.device('cuda', 0)
ctx = brotli_amd.DeviceContext(0, profiling=True)
k, size = (1024, 1 << 20) if not os.environ.get('REF_ONLY') else (16, 1 << 20)
data = datagen.enwik_device(k * size, 2000, dev)
cap = k * size + k * 8192
comp = torch.empty(cap, dtype=torch.uint8, device=dev)
off = ctx.encode(data.data_ptr(), [i * size for i in range(k + 1)], comp.data_ptr(), cap, {'quality': 11})
slot = size + 4096
dec = torch.empty(k * slot, dtype=torch.uint8, device=dev)
out_dir = os.path.join(ROOT, 'gpurun_out', 'c4_sample')
os.makedirs(out_dir, exist_ok=True)
raw = comp[:off[-1]].cpu().numpy().tobytes()
host = data[:16 * size].cpu().numpy().tobytes()
for i in range(16):
    with open(os.path.join(out_dir, '%02d.br' % i), 'wb') as f:
        f.write(raw[off[i]:off[i + 1]])
    with open(os.path.join(out_dir, '%02d.bin' % i), 'wb') as f:
        f.write(host[i * size:(i + 1) * size])
counters(1)
for it in range(0 if os.environ.get('REF_ONLY') else 2):
    sizes, st = ctx.decode(comp.data_ptr(), off, dec.data_ptr(), [i * slot for i in range(k + 1)])
    ok = torch.equal(dec.view(k, slot)[:, :size], data.view(k, size))
    print('c4', it, ctx.kernel_times(), 'ok' if ok else 'MISMATCH', counters(k), flush=True)

gold = os.path.join(ROOT, 'tests', 'golden', 'bench')
for name in ('noto-tc', 'enc-ttf', 'html-content'):
    enc = open(os.path.join(gold, name + '.br'), 'rb').read()
    n = len(brotli_amd.brotliDecode(enc))
    src = torch.tensor(list(enc), dtype=torch.uint8, device=dev)
    o = torch.empty(n + 4096, dtype=torch.uint8, device=dev)
    counters(1)
    ctx.decode(src.data_ptr(), [0, len(enc)], o.data_ptr(), [0, n + 4096])
    print(name, len(enc), n, ctx.kernel_times(), counters(1), flush=True)
