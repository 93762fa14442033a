"""Find enwik_device buffers (bench c4 input) whose oracle encode does not round-trip."""
import os, sys
from concurrent.futures import ThreadPoolExecutor
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'tests')); sys.path.insert(0, os.path.join(ROOT, 'brotli-lib_amd', 'python'))
import torch, _oracle
from brotli_amd import datagen
n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
d = datagen.enwik_device(n << 20, 2000, torch.device('cuda', 0)).cpu().numpy().tobytes()
def one(i):
    b = d[i << 20:(i + 1) << 20]
    e = _oracle.encode(b, 11, 22, 0)
    r = _oracle.decode(e)
    ok = r == b
    if not ok:
        os.makedirs(os.path.join(ROOT, 'gpurun_out', 'fail'), exist_ok=True)
        open(os.path.join(ROOT, 'gpurun_out', 'fail', 'in_%d.bin' % i), 'wb').write(b)
    return i, ok, r if isinstance(r, int) else -999
with ThreadPoolExecutor(16) as ex:
    res = list(ex.map(one, range(n)))
print([r for r in res if not r[1]], flush=True)
