"""Overlap probe (C4 shape): does decoding batch i on one context while batch i+1 encodes on
another fill the GPU better than running them back to back?  Prints one JSON line per mode.
MIB_DEC_GRID caps the decoder's persistent grid (fewer decoder waves per CU leave LDS for the
encoder's kernels)."""
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'brotli-lib_amd', 'python'))
import torch  # noqa: E402
import brotli_amd  # noqa: E402
from brotli_amd import datagen  # noqa: E402

k, size = int(os.environ.get('K', '1024')), 1 << 20
dev = torch.device('cuda', 0)
data = datagen.enwik_device(k * size, 2000, dev)
in_off = [i * size for i in range(k + 1)]
cap = k * size + k * size // 8 + 4096 * k
comp = [torch.empty(cap, dtype=torch.uint8, device=dev) for _ in range(2)]
slot = size + 4096
dec = torch.empty(k * slot, dtype=torch.uint8, device=dev)
dec_off = [i * slot for i in range(k + 1)]
ce, cd = brotli_amd.DeviceContext(0), brotli_amd.DeviceContext(0)
opts = {'quality': 11}
off = [ce.encode(data.data_ptr(), in_off, comp[b].data_ptr(), cap, opts) for b in range(2)]
cd.decode(comp[0].data_ptr(), off[0], dec.data_ptr(), dec_off)
torch.cuda.synchronize()
assert torch.equal(dec.view(k, slot)[:, :size], data.view(k, size))
n = int(os.environ.get('N', '3'))

t = time.perf_counter()
for i in range(n):
    ce.encode(data.data_ptr(), in_off, comp[i & 1].data_ptr(), cap, opts)
    cd.decode(comp[i & 1].data_ptr(), off[i & 1], dec.data_ptr(), dec_off)
torch.cuda.synchronize()
serial = (time.perf_counter() - t) / n
t = time.perf_counter()
for i in range(n):
    cd.decode(comp[0].data_ptr(), off[0], dec.data_ptr(), dec_off)
torch.cuda.synchronize()
dec_only = (time.perf_counter() - t) / n

# pipelined: encode of batch i+1 (context ce) beside decode of batch i (context cd)
res = {}


def enc_loop():
    for i in range(n):
        ce.encode(data.data_ptr(), in_off, comp[(i + 1) & 1].data_ptr(), cap, opts)


def dec_loop():
    for i in range(n):
        cd.decode(comp[i & 1].data_ptr(), off[i & 1], dec.data_ptr(), dec_off)


t = time.perf_counter()
a, b = threading.Thread(target=enc_loop), threading.Thread(target=dec_loop)
a.start(); b.start(); a.join(); b.join()
torch.cuda.synchronize()
pipe = (time.perf_counter() - t) / n
ok = torch.equal(dec.view(k, slot)[:, :size], data.view(k, size))
print(json.dumps({'dec_grid': os.environ.get('MIB_DEC_GRID'), 'serial_ms': round(serial * 1e3, 1),
                  'dec_only_ms': round(dec_only * 1e3, 1), 'pipelined_ms': round(pipe * 1e3, 1),
                  'serial_MBps': round(k * size / 1e6 / serial, 1), 'pipelined_MBps': round(k * size / 1e6 / pipe, 1),
                  'ok': ok}), flush=True)
