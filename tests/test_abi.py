"""CPU-side checks of the drop-in boundary: the in-tree library loads and exports every
entry point include/brotli_amd.h declares; the host mirror keeps the reference's surface."""
import ctypes
import os
import re

import brotli_amd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    with open(os.path.join(ROOT, 'include', 'brotli_amd.h')) as f:
        src = f.read()
    src = re.sub(r'/\*.*?\*/', '', src, flags=re.S)
    return sorted(set(re.findall(r'\b(mib_[a-z0-9_]+)\s*\(', src)))


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(brotli_amd.library_path())
    names = declared_functions()
    assert len(names) >= 19
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_host_mirror_surface():
    for name in ('brotliEncode', 'BrotliEncoder', 'brotliDecode', 'brotliDecodedSize', 'EncoderMode'):
        assert hasattr(brotli_amd, name)
    assert (brotli_amd.EncoderMode.GENERIC, brotli_amd.EncoderMode.TEXT, brotli_amd.EncoderMode.FONT) == (0, 1, 2)


def test_decoded_size_is_header_only():
    # brotliDecodedSize parses the first metablock header (engine.ts:2155-2192): no device needed
    import _oracle
    for nm in sorted(os.listdir(os.path.join(ROOT, 'tests', 'golden', 'vectors'))):
        if '.compressed' in nm:
            with open(os.path.join(ROOT, 'tests', 'golden', 'vectors', nm), 'rb') as f:
                b = f.read()
            assert brotli_amd.brotliDecodedSize(b) == _oracle.peek_size(b), nm


def test_strerror_matches_reference_messages():
    lib = ctypes.CDLL(brotli_amd.library_path())
    lib.mib_strerror.restype = ctypes.c_char_p
    assert lib.mib_strerror(-9) == b'Brotli error code: -9'
    assert lib.mib_strerror(-30) == b'Brotli error code: -30'
