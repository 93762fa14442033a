"""C3 decoder diagnostics (MIB_PROF build via BROTLI_AMD_LIB): 64 WOFF2-glyf buffers encoded in
FONT mode (MIB_CTX_MODE may force the literal context mode), then decoded with the phase and
table-placement counters: metablocks whose prefix-code tables fit the LDS area vs HBM."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'brotli-lib_amd', 'python'))
import brotli_amd  # noqa: E402
from brotli_amd import datagen  # noqa: E402

NAMES = ['cmd_tail', 'lit_tail', 'distance', 'copy_rest', 'n_literals', 'n_commands', 'mb_lds_tables', 'mb_hbm_tables',
         'F_cmd', 'F_lit', 'F_dist', 'F_copy', 'F_top', 'copy_readlane', 'fast_cmds', 'fast_calls']
lib = brotli_amd._L()
prof = (ctypes.c_ulonglong * 16)()
k = int(os.environ.get('K', '64'))
bufs = datagen.glyf_font_batch(k, 262144, 1000, workers=8)
outs = brotli_amd.encode_batch(bufs, {'quality': 11, 'mode': 2})
lib.mib_debug_read_prof(prof)
dec = brotli_amd.decode_batch(outs)
assert dec == bufs
lib.mib_debug_read_prof(prof)
print('mode', os.environ.get('MIB_CTX_MODE', 'default'), 'ratio %.5f' % (sum(map(len, outs)) / (k * 262144)),
      {n: round(v / k, 1) for n, v in zip(NAMES, prof)}, flush=True)
