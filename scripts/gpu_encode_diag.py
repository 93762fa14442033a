"""Staged GPU encoder check: small cases first, printing progress to gpurun_out/enc_diag.log."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'brotli-lib_amd', 'python'))
sys.path.insert(0, os.path.join(ROOT, 'tests'))
import brotli_amd  # noqa: E402
import _oracle  # noqa: E402
from brotli_amd import datagen  # noqa: E402

log = open(os.path.join(ROOT, 'gpurun_out', 'enc_diag.log'), 'w')


def P(*a):
    print(*a, file=log, flush=True)


def check(name, data, opts=None):
    t = time.time()
    enc = brotli_amd.brotliEncode(data, opts or {})
    dt = time.time() - t
    o = _oracle.decode(enc)
    ok = isinstance(o, bytes) and o == data
    g = brotli_amd.brotliDecode(enc) if ok else None
    P('%-28s n=%-9d enc=%-9d %.3fs oracle_ok=%s gpu_ok=%s' % (name, len(data), len(enc), dt, ok, g == data))
    if not ok:
        P('  oracle result:', o if not isinstance(o, bytes) else 'mismatch len %d' % len(o))
        P('  head:', enc[:64].hex())
    return ok


cases = [('empty', b''), ('one', b'a'), ('63', b'x' * 63), ('fox64', datagen.fox(2)[:64]), ('fox', datagen.fox(200)),
         ('text100k', datagen.enwik_text(100000, 1)), ('zeros200k', b'\0' * 200000),
         ('rand100k', datagen.random_bytes(100000, datagen.xorshift32(5))), ('text1M', datagen.enwik_text(1 << 20, 2))]
allok = True
for nm, d in cases:
    allok &= check(nm, d)
c = brotli_amd.DeviceContext(0, profiling=True)
import torch  # noqa: E402
d = datagen.enwik_text(1 << 20, 3)
bufs = [d] * 64
x = torch.frombuffer(bytearray(b''.join(bufs)), dtype=torch.uint8).cuda()
out = torch.empty(len(d) * 64 * 2, dtype=torch.uint8, device='cuda')
offs = [i * len(d) for i in range(65)]
for it in range(3):
    torch.cuda.synchronize()
    t = time.time()
    oo = c.encode(x.data_ptr(), offs, out.data_ptr(), out.numel())
    torch.cuda.synchronize()
    P('ctx encode 64x1MiB: %.3fs  -> %d bytes; %s' % (time.time() - t, oo[-1], sorted(c.kernel_times().items())))
e0 = out[:oo[1]].cpu().numpy().tobytes()
P('ctx stream 0 decodes:', _oracle.decode(e0) == d)
P('ALL OK' if allok else 'FAILURES')
sys.exit(0 if allok else 1)
