"""ctypes binding of the ORACLE (oracle/liboracle.so): the CPU restatement of the
reference used as the checker.  Test infrastructure only -- the product never imports it."""
import ctypes
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, 'oracle', 'liboracle.so')
_lib = None
_P = ctypes.POINTER(ctypes.c_uint8)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            subprocess.run(['make', '-s', '-C', os.path.join(ROOT, 'oracle')], check=True)
        _lib = ctypes.CDLL(LIB)
        _lib.oracle_encode.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                       ctypes.POINTER(_P), ctypes.POINTER(ctypes.c_size_t)]
        _lib.oracle_decode.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t,
                                       ctypes.c_int64, ctypes.POINTER(_P), ctypes.POINTER(ctypes.c_size_t)]
        _lib.oracle_peek_decoded_size.argtypes = [ctypes.c_char_p, ctypes.c_size_t]
        _lib.oracle_peek_decoded_size.restype = ctypes.c_int64
    return _lib


def encode(data, quality=11, lgwin=22, mode=0):
    """oracle brotliEncode (ref-fixed); raises on unsupported quality."""
    o, n = _P(), ctypes.c_size_t()
    rc = lib().oracle_encode(data, len(data), quality, lgwin, mode, ctypes.byref(o), ctypes.byref(n))
    if rc:
        raise RuntimeError('oracle_encode rc=%d' % rc)
    r = ctypes.string_at(o, n.value)
    lib().oracle_free(o)
    return r


def peek_size(data):
    return lib().oracle_peek_decoded_size(data, len(data))


def decode(data, out_size=None, dictionary=None):
    """oracle engine brotliDecode: returns bytes, or the negative reference error code (int)."""
    if out_size is None:
        p = peek_size(data)
        out_size = p if p > 0 else -1
    o, n = _P(), ctypes.c_size_t()
    d = bytes(dictionary) if dictionary is not None else None   # an empty dictionary is still attached
    rc = lib().oracle_decode(data, len(data), d, len(d) if d is not None else 0, out_size, ctypes.byref(o),
                             ctypes.byref(n))
    if rc:
        return rc
    r = ctypes.string_at(o, n.value)
    lib().oracle_free(o)
    return r
