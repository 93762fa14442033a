"""C5 host-side time split (GPU box): where the streaming encode's and the 1 GiB decode's wall
time goes outside the kernels.  Prints one JSON line.

  python3 scripts/c5_host_diag.py            (SIZE env: stream bytes, default 1 GiB)
"""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'brotli-lib_amd', 'python'))

import torch  # noqa: E402
import brotli_amd  # noqa: E402
from brotli_amd import datagen  # noqa: E402

MIB = 1 << 20


def main():
    size = int(os.environ.get('SIZE', str(1 << 30)))
    dev = torch.device('cuda', 0)
    data = datagen.c5_stream(size, 5000, dev)
    cdict = datagen.c5_dictionary()
    opts = {'quality': 9, 'lgwin': 24, 'mode': 1, 'customDictionary': cdict}
    res = {}

    def enc(slicer, tag):
        e = brotli_amd.BrotliEncoder(opts)
        t_slice = t_fill = t_run = 0.0
        nrun = 0
        parts = []
        t0 = time.perf_counter()
        for p in range(0, size, MIB):
            a = time.perf_counter()
            ch = slicer(p)
            b = time.perf_counter()
            out = e.update(ch)
            c = time.perf_counter()
            t_slice += b - a
            if out:
                t_run += c - b
                nrun += 1
            else:
                t_fill += c - b
            parts.append(out)
        a = time.perf_counter()
        parts.append(e.finish())
        t_fin = time.perf_counter() - a
        a = time.perf_counter()
        s = b''.join(parts)
        t_join = time.perf_counter() - a
        res[tag] = dict(total_ms=1e3 * (time.perf_counter() - t0), slice_ms=1e3 * t_slice,
                        fill_ms=1e3 * t_fill, run_ms=1e3 * t_run, runs=nrun, finish_ms=1e3 * t_fin,
                        join_ms=1e3 * t_join)
        return s

    mv = memoryview(data)
    stream = enc(lambda p: data[p:p + MIB], 'warm')
    brotli_amd.default_profiling(True)
    stream = enc(lambda p: data[p:p + MIB], 'enc_bytes_slices')
    kt = brotli_amd.default_kernel_times()
    res['enc_kernel_ms'] = sum(v[0] for v in kt.values())
    brotli_amd.default_profiling(False)
    enc(lambda p: mv[p:p + MIB], 'enc_memoryview_slices')

    # decode: the C call (H2D, kernels, D2H into malloc) and the copy into a Python bytes
    L = brotli_amd._L()
    for rep in range(4):
        os.environ['MIB_PY_HUGEPAGE'] = '0' if rep < 2 else '1'
        brotli_amd.default_profiling(True)
        buf = brotli_amd._Buf()
        a = time.perf_counter()
        rc = L.mib_decode(stream, len(stream), cdict, len(cdict), -1, -1, ctypes.byref(buf))
        b = time.perf_counter()
        out = brotli_amd._take(buf)
        c = time.perf_counter()
        kt = brotli_amd.default_kernel_times()
        brotli_amd.default_profiling(False)
        assert rc == 0 and out == data
        res['dec%d' % rep] = dict(c_call_ms=1e3 * (b - a), take_ms=1e3 * (c - b),
                                  kernel_ms=sum(v[0] for v in kt.values()))
        del out
    res['stream_bytes'] = len(stream)

    # PCIe and host-memory rates for the same 1 GiB: pageable and pinned, H2D and D2H
    g = torch.empty(size, dtype=torch.uint8, device=dev)
    h = torch.frombuffer(bytearray(data), dtype=torch.uint8)
    hp = torch.empty(size, dtype=torch.uint8).pin_memory()
    for name, fn in (('h2d_pageable', lambda: g.copy_(h)), ('h2d_pinned', lambda: g.copy_(hp)),
                     ('d2h_pageable', lambda: h.copy_(g)), ('d2h_pinned', lambda: hp.copy_(g)),
                     ('host_memcpy', lambda: h.copy_(hp)),
                     ('bytes_from_fresh', lambda: bytes(memoryview(data)[:size]))):
        fn()
        torch.cuda.synchronize()
        a = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        res[name + '_GBps'] = size / (time.perf_counter() - a) / 1e9
    print(json.dumps(res))


if __name__ == '__main__':
    main()
