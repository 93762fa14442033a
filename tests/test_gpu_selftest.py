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
