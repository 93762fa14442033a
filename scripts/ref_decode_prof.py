"""Decoder phase counters (MIB_PROF build: BROTLI_AMD_LIB=brotli-lib_amd/libbrotli_amd_prof.so)
on the reference's own bench streams, one stream per call (the `ref` bench leg's shape)."""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'brotli-lib_amd', 'python'))
import torch  # noqa: E402,F401
import brotli_amd  # noqa: E402

NAMES = ['cmd_tail', 'lit_tail', 'distance', 'copy_rest', 'n_literals', 'n_commands', 'mb_lds_tables',
         'mb_hbm_tables', 'F_cmd', 'F_lit', 'F_dist', 'F_copy', 'F_top', 'copy_readlane', 'fast_cmds', 'fast_calls']
lib = brotli_amd._L()
prof = (ctypes.c_ulonglong * 16)()
has = hasattr(lib, 'mib_debug_read_prof')
for name in os.environ.get('STREAMS', 'noto-tc,enc-ttf').split(','):
    d = open(os.path.join(ROOT, 'tests', 'golden', 'bench', name + '.br'), 'rb').read()
    out = brotli_amd.brotliDecode(d)
    if has:
        lib.mib_debug_read_prof(prof)
    brotli_amd.default_profiling(True)
    t = time.perf_counter()
    out = brotli_amd.brotliDecode(d)
    ms = 1e3 * (time.perf_counter() - t)
    kt = brotli_amd.default_kernel_times()
    brotli_amd.default_profiling(False)
    line = {'stream': name, 'out': len(out), 'wall_ms': round(ms, 2), 'kernels': kt}
    if has:
        lib.mib_debug_read_prof(prof)
        line['prof'] = dict(zip(NAMES, list(prof)))
    print(line, flush=True)
