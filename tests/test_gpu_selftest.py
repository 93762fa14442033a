"""Hardware properties the HIP kernels rely on, checked on the MI355X itself."""
import ctypes

import pytest

import brotli_amd

pytestmark = pytest.mark.gpu


def test_lds_atomics_serve_lanes_in_order():
    """enc_sort.hip ranks a wave's items by returning LDS atomics: equal digits must get their
    slots in lane order, or the per-bucket chains of the match finder lose their position
    order (scripts/probe/lds_atomic_order.hip is the stand-alone probe)."""
    lib = brotli_amd._L()
    lib.mib_selftest_lds_atomic_order.restype = ctypes.c_int64
    lib.mib_selftest_lds_atomic_order.argtypes = [ctypes.c_int]
    assert lib.mib_selftest_lds_atomic_order(1 << 15) == 0


def test_ballot_ranked_sort_gives_the_same_streams():
    """The fallback the library takes on a device that fails the self-test above (ensure_device,
    runtime.cpp): the bucket sort ranks by wave ballots, which need no atomic order, and must give
    the same stable order -- so the same stream bytes -- as the fast ranking."""
    from brotli_amd import datagen
    lib = brotli_amd._L()
    lib.mib_force_ballot_rank.restype = None
    lib.mib_force_ballot_rank.argtypes = [ctypes.c_int]
    d = datagen.enwik_text(8 << 20, 77)
    bufs = [d[i:i + (1 << 20)] for i in range(0, len(d), 1 << 20)] + [d[:300000]]
    for mode in (0, 2):
        opts = {'quality': 11, 'mode': mode}
        fast = brotli_amd.encode_batch(bufs, opts)
        lib.mib_force_ballot_rank(1)
        try:
            slow = brotli_amd.encode_batch(bufs, opts)
        finally:
            lib.mib_force_ballot_rank(0)
        assert slow == fast
    assert brotli_amd.decode_batch(fast) == bufs
