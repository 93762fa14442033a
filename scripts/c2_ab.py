"""C2 A/B: encode the 64 MiB C2 buffer with the library BROTLI_AMD_LIB points at, write the
stream to gpurun_out/c2_<tag>.br and report the oracle's and the HIP decoder's verdicts."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'brotli-lib_amd', 'python'))
sys.path.insert(0, os.path.join(ROOT, 'tests'))
import brotli_amd  # noqa: E402
from brotli_amd import datagen  # noqa: E402
import _oracle  # noqa: E402

tag = sys.argv[1]
d = datagen.enwik_text(64 << 20, 2)
enc = brotli_amd.brotliEncode(d, {'quality': 11, 'lgwin': 22})
open(os.path.join(ROOT, 'gpurun_out', 'c2_%s.br' % tag), 'wb').write(enc)
got = _oracle.decode(enc)
print(tag, len(enc), 'oracle', 'ok' if got == d else got if not isinstance(got, bytes) else 'mismatch',
      'hip', 'ok' if brotli_amd.brotliDecode(enc) == d else 'bad', flush=True)
