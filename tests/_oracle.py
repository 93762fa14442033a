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


def bt_matches(data, lgwin=22):
    """per-position findAllMatches lists (pass 1 of the q11 parse): [(i, [(distance, length)...])]"""
    import array
    cap = 8 * len(data) + 64
    buf = (ctypes.c_uint32 * cap)()
    lib().oracle_bt_matches.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t]
    lib().oracle_bt_matches.restype = ctypes.c_int64
    w = lib().oracle_bt_matches(data, len(data), lgwin, buf, cap)
    if w < 0:
        raise RuntimeError('oracle_bt_matches: output too small')
    v = array.array('I', bytes(buf)[:4 * w])
    out, k = [], 0
    while k < w:
        i, c = v[k], v[k + 1]
        out.append((i, [(v[k + 2 + 2 * q], v[k + 3 + 2 * q]) for q in range(c)]))
        k += 2 + 2 * c
    return out


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


PROBE_DTYPE = None


def word_refs():
    """static-dictionary word references the oracle decoder has met in this process"""
    lib().oracle_word_refs.restype = ctypes.c_uint64
    return lib().oracle_word_refs()


def compound_refs():
    """compound-dictionary (customDictionary) copies the oracle decoder has met in this process"""
    lib().oracle_compound_refs.restype = ctypes.c_uint64
    return lib().oracle_compound_refs()


def dist_code_counts():
    """copies the oracle decoder has decoded on this thread since the last call, by distance
    code: [implicit (command code < 128), code 0, short codes 1-15, explicit distances]"""
    out = (ctypes.c_uint64 * 4)()
    lib().oracle_dist_code_counts(out)
    return list(out)


def probe(data, positions):
    """decoder states (parts.h PartEntry layout) at the given ascending output positions:
    the command starting there, or the metablock header starting there (flags bit 2)."""
    import numpy as np
    from _parts import ENTRY_DTYPE
    pos = np.ascontiguousarray(np.asarray(positions, dtype=np.uint64))
    out = np.zeros(len(pos), dtype=ENTRY_DTYPE)
    f = lib().oracle_decode_probe
    f.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
    rc = f(data, len(data), pos.ctypes.data, len(pos), out.ctypes.data)
    if rc:
        raise RuntimeError('oracle_decode_probe rc=%d' % rc)
    return out


def max_block_types():
    """the largest (literal, command, distance) block type counts of any metablock the oracle
    decoder has decoded on this thread since the last call"""
    out = (ctypes.c_int * 3)()
    lib().oracle_max_block_types(out)
    return list(out)
