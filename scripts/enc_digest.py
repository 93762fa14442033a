"""SHA-256 of the encoder's output on fixed inputs, for comparing two library builds
(BROTLI_AMD_LIB) byte for byte: C4's shape (64 x 1 MiB text, q11), C3's (64 x 256 KiB glyf,
FONT), C2's (one 64 MiB stream), and the reference's update() cadence (16 x 1 MiB, q9 lgwin 24).
usage: python3 scripts/enc_digest.py > digest.json"""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'brotli-lib_amd', 'python'))
import torch  # noqa: E402
import brotli_amd  # noqa: E402
import bench  # noqa: E402
from brotli_amd import datagen  # noqa: E402

dev = torch.device('cuda', 0)
ctx = brotli_amd.DeviceContext(0)
out = {}
for wl, k in (('c4', 64), ('c3', 64), ('c2', 1)):
    _, size, mode, _, _ = bench.WORKLOADS[wl]
    data = bench.make_inputs(wl, k, size, 0, dev)
    cap = k * size + k * size // 8 + 4096 * k
    comp = torch.empty(cap, dtype=torch.uint8, device=dev)
    off = ctx.encode(data.data_ptr(), [i * size for i in range(k + 1)], comp.data_ptr(), cap, {'quality': 11, 'mode': mode})
    torch.cuda.synchronize()
    b = comp[:off[-1]].cpu().numpy().tobytes()
    out[wl] = [off[-1], hashlib.sha256(b).hexdigest()[:16]]
    print(wl, out[wl], file=sys.stderr, flush=True)
text = datagen.enwik_text(16 << 20, 3)
enc = brotli_amd.BrotliEncoder({'quality': 9, 'lgwin': 24})
parts = [enc.update(text[i << 20:(i + 1) << 20]) for i in range(16)]
parts.append(enc.finish())
b = b''.join(parts)
out['cadence'] = [len(b), hashlib.sha256(b).hexdigest()[:16]]
print(json.dumps(out))
