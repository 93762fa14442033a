"""Host-transfer probe (round 5): what one GiB costs each way on this box --
torch pinned copies (the PCIe rate), a numpy copy from pinned memory into fresh bytes objects
(the host side of the ring), and the library's batch calls on C4's shape with the experiment
build's MIB_HOST_TIMING phase times (stderr)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'brotli-lib_amd', 'python'))
import numpy as np  # noqa: E402
import torch  # noqa: E402

dev = torch.device('cuda', 0)
n = 1 << 30
d = torch.empty(n, dtype=torch.uint8, device=dev)
d.fill_(7)
pin = torch.empty(n, dtype=torch.uint8, pin_memory=True)
res = {}
for it in range(2):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    pin.copy_(d, non_blocking=True)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    d.copy_(pin, non_blocking=True)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    res['d2h_pinned_GBps'] = round(n / 1e9 / (t1 - t0), 2)
    res['h2d_pinned_GBps'] = round(n / 1e9 / (t2 - t1), 2)
src = pin.numpy()
for it in range(2):
    t0 = time.perf_counter()
    outs = [bytearray(src[i << 20:(i + 1) << 20]) for i in range(1024)]
    t1 = time.perf_counter()
    res['host_copy_1thread_into_new_GBps'] = round(n / 1e9 / (t1 - t0), 2)
    del outs
print(json.dumps(res), flush=True)
del d, pin, src
import brotli_amd  # noqa: E402
from brotli_amd import datagen  # noqa: E402
data = datagen.enwik_device(n, 0, dev).cpu().numpy().tobytes()
bufs = [data[i << 20:(i + 1) << 20] for i in range(1024)]
del data
gpus = int(os.environ.get('PROBE_GPUS', '0')) or None
for it in range(3):
    t0 = time.perf_counter()
    comp = brotli_amd.encode_batch(bufs, {'quality': 11, 'lgwin': 22}, gpus=gpus)
    t1 = time.perf_counter()
    out = brotli_amd.decode_batch(comp, gpus=gpus)
    t2 = time.perf_counter()
    del out
    t3 = time.perf_counter()
    out = brotli_amd.decode_batch(comp, gpus=gpus)
    t4 = time.perf_counter()
    print(json.dumps({'iter': it, 'decode_again_ms': round((t4 - t3) * 1e3, 1), 'free_ms': round((t3 - t2) * 1e3, 1)}), flush=True)
    print(json.dumps({'iter': it, 'encode_ms': round((t1 - t0) * 1e3, 1), 'decode_ms': round((t2 - t1) * 1e3, 1),
                      'ok': out == bufs}), flush=True)
    sys.stderr.flush()
