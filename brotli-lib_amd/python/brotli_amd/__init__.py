"""Python mirror of countertype/brotli-lib's public API over the brotli_amd C ABI.

    brotliEncode(input, options)   src/encode/encode.ts:50-90
    BrotliEncoder(options)         src/encode/encode.ts:290-490
    brotliDecode(data, options)    src/decode/decode.ts:18-65   (options dict or legacy int)
    brotliDecodedSize(data)        src/decode/decode.ts:9-11
    EncoderMode                    src/encode/enc-constants.ts:56-60

Same argument meaning and error behaviour as the reference: decoder failures raise
``BrotliError("Brotli error code: N")`` with the reference's N, ``maxOutputSize`` raises
``BrotliError("Decompressed size X exceeds limit Y")``.  All compute runs in the HIP
library (libbrotli_amd.so, built in-tree by __graft_entry__.build()); there is no CPU
fallback -- without an MI355X the calls raise.
"""
import ctypes
import os

__all__ = ['brotliEncode', 'BrotliEncoder', 'brotliDecode', 'brotliDecodedSize', 'EncoderMode', 'BrotliError',
           'encode_batch', 'decode_batch', 'encoder_update_batch', 'DeviceContext', 'library_path']

_PKG = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
# BROTLI_AMD_LIB: an instrumented build of the same library (timing experiments only)
_LIB_PATH = os.environ.get('BROTLI_AMD_LIB') or os.path.join(_PKG, 'libbrotli_amd.so')


def library_path():
    return _LIB_PATH


class EncoderMode:
    GENERIC = 0
    TEXT = 1
    FONT = 2


class BrotliError(Exception):
    def __init__(self, message, code=None):
        super().__init__(message)
        self.code = code


class _Opts(ctypes.Structure):
    _fields_ = [('quality', ctypes.c_int), ('lgwin', ctypes.c_int), ('mode', ctypes.c_int),
                ('size_hint', ctypes.c_uint64), ('dict', ctypes.c_char_p), ('dict_len', ctypes.c_uint64),
                ('stream_chunk', ctypes.c_uint64)]


class _Buf(ctypes.Structure):
    _fields_ = [('data', ctypes.POINTER(ctypes.c_uint8)), ('size', ctypes.c_size_t)]


class _Span(ctypes.Structure):
    _fields_ = [('data', ctypes.c_void_p), ('size', ctypes.c_size_t)]


class _KTime(ctypes.Structure):
    _fields_ = [('name', ctypes.c_char * 32), ('ms', ctypes.c_double), ('launches', ctypes.c_uint32)]


_lib = None

# Results come back as bytes objects the library writes into (mib_set_allocator): the device
# copies its output straight into the object returned, no copy through a C buffer.
_ALLOC_FN = ctypes.CFUNCTYPE(ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t)
_FREE_FN = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_void_p)
_new_bytes = ctypes.pythonapi.PyBytes_FromStringAndSize
_new_bytes.restype = ctypes.py_object
_new_bytes.argtypes = [ctypes.c_char_p, ctypes.c_ssize_t]
_results = {}   # address -> the bytes object the library is filling / has filled
_HUGE = 2 << 20
_madvise = ctypes.CDLL(None, use_errno=True).madvise
_madvise.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]


def _alloc(opaque, size):
    try:
        b = _new_bytes(None, max(1, size))   # (a fresh object: b'' is a shared singleton)
    except MemoryError:
        return None
    addr = ctypes.cast(ctypes.c_char_p(b), ctypes.c_void_p).value
    _results[addr] = b
    if size >= _HUGE and os.environ.get('MIB_PY_HUGEPAGE') != '0':
        # large results: the copy into fresh memory is page-fault bound; 2 MiB pages fault 512x less
        lo = (addr + _HUGE - 1) & ~(_HUGE - 1)
        hi = (addr + size) & ~(_HUGE - 1)
        if hi > lo:
            _madvise(lo, hi - lo, 14)   # MADV_HUGEPAGE
    return addr


def _free(opaque, addr):
    _results.pop(addr, None)


_alloc_cb = _ALLOC_FN(_alloc)
_free_cb = _FREE_FN(_free)


def _L():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            raise BrotliError('brotli_amd: %s not built (run __graft_entry__.build())' % _LIB_PATH)
        # PyTorch-ROCm ships its own libamdhip64 (same soname).  Loading torch first makes the
        # library bind to that one runtime; the other order would put two HIP runtimes in the
        # process and torch's device init would fail.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        lib = ctypes.CDLL(_LIB_PATH)
        u8p = ctypes.c_char_p
        lib.mib_strerror.restype = ctypes.c_char_p
        lib.mib_strerror.argtypes = [ctypes.c_int]
        lib.mib_init.argtypes = [ctypes.c_int]
        lib.mib_encode.argtypes = [u8p, ctypes.c_size_t, ctypes.POINTER(_Opts), ctypes.POINTER(_Buf)]
        lib.mib_decode.argtypes = [u8p, ctypes.c_size_t, u8p, ctypes.c_size_t, ctypes.c_int64, ctypes.c_int64,
                                   ctypes.POINTER(_Buf)]
        lib.mib_decoded_size.argtypes = [u8p, ctypes.c_size_t]
        lib.mib_decoded_size.restype = ctypes.c_int64
        lib.mib_buf_free.argtypes = [ctypes.POINTER(_Buf)]
        lib.mib_encoder_new.argtypes = [ctypes.POINTER(_Opts)]
        lib.mib_encoder_new.restype = ctypes.c_void_p
        lib.mib_encoder_update.argtypes = [ctypes.c_void_p, u8p, ctypes.c_size_t, ctypes.POINTER(_Buf)]
        lib.mib_encoder_finish.argtypes = [ctypes.c_void_p, ctypes.POINTER(_Buf)]
        lib.mib_encoder_free.argtypes = [ctypes.c_void_p]
        lib.mib_encoder_update_batch.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(_Span), ctypes.c_size_t,
                                                 ctypes.POINTER(_Buf)]
        lib.mib_encode_batch.argtypes = [ctypes.POINTER(_Span), ctypes.c_size_t, ctypes.POINTER(_Opts),
                                         ctypes.POINTER(_Buf), ctypes.POINTER(ctypes.c_int)]
        lib.mib_decode_batch.argtypes = [ctypes.POINTER(_Span), ctypes.c_size_t, ctypes.POINTER(_Buf),
                                         ctypes.POINTER(ctypes.c_int)]
        lib.mib_encode_batch_n.argtypes = [ctypes.POINTER(_Span), ctypes.c_size_t, ctypes.POINTER(_Opts), ctypes.c_int,
                                           ctypes.POINTER(_Buf), ctypes.POINTER(ctypes.c_int)]
        lib.mib_decode_batch_n.argtypes = [ctypes.POINTER(_Span), ctypes.c_size_t, ctypes.c_int, ctypes.POINTER(_Buf),
                                           ctypes.POINTER(ctypes.c_int)]
        lib.mib_ctx_new.argtypes = [ctypes.c_int]
        lib.mib_ctx_new.restype = ctypes.c_void_p
        lib.mib_ctx_free.argtypes = [ctypes.c_void_p]
        lib.mib_ctx_encode.argtypes = [ctypes.c_void_p, ctypes.POINTER(_Opts), ctypes.c_void_p,
                                       ctypes.POINTER(ctypes.c_uint64), ctypes.c_size_t, ctypes.c_void_p,
                                       ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64), ctypes.c_void_p]
        lib.mib_ctx_decode.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64),
                                       ctypes.c_size_t, ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64),
                                       ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int), ctypes.c_void_p]
        lib.mib_ctx_kernel_times.argtypes = [ctypes.c_void_p, ctypes.POINTER(_KTime), ctypes.c_int]
        lib.mib_ctx_set_profiling.argtypes = [ctypes.c_void_p, ctypes.c_int]
        lib.mib_woff2_transform_glyf.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(_Buf)]
        lib.mib_woff2_transform_hmtx.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(_Buf)]
        lib.mib_part_stats.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]
        lib.mib_default_ctx.restype = ctypes.c_void_p
        lib.mib_ctx_clear_times.argtypes = [ctypes.c_void_p]
        lib.mib_set_allocator.argtypes = [_ALLOC_FN, _FREE_FN, ctypes.c_void_p]
        lib.mib_set_allocator(_alloc_cb, _free_cb, None)
        _lib = lib
    return _lib


def _err(code, what=''):
    msg = _L().mib_strerror(code).decode()
    return BrotliError(msg, code)


def _take(buf):
    addr = ctypes.cast(buf.data, ctypes.c_void_p).value
    b = _results.pop(addr, None) if addr else None
    if b is None:
        return b''
    buf.data = None
    return b if len(b) == buf.size else b[:buf.size]


def _opts(options):
    """option clamping of encode.ts:54-71 / BrotliEncoder constructor :293-310; plus the
    extension `customDictionary` (the encoder side of brotliDecode's option of that name:
    the stream then decodes with, and only with, the same dictionary).  The dictionary's
    bytes object is kept on the returned structure for the duration of the call."""
    options = options or {}
    o = _Opts(11, 22, EncoderMode.GENERIC, 0, None, 0, 0)
    if options.get('quality') is not None:
        o.quality = max(0, min(11, int(options['quality'])))
    if options.get('lgwin') is not None:
        o.lgwin = max(10, min(24, int(options['lgwin'])))
    if options.get('mode') is not None:
        o.mode = int(options['mode'])
    if options.get('sizeHint') is not None:
        o.size_hint = int(options['sizeHint'])
    if options.get('streamChunk') is not None:   # BrotliEncoder throughput mode (brotli_amd.h)
        o.stream_chunk = max(0, int(options['streamChunk']))
    if options.get('customDictionary') is not None:
        d = _bytes(options['customDictionary'])
        o._keep = d
        o.dict, o.dict_len = d, len(d)
    return o


def _in(x):
    """(argument, length, keep-alive) for an input buffer, without copying it: bytes as is,
    any other C-contiguous buffer (bytearray, memoryview slices, numpy, array) by address."""
    if isinstance(x, bytes):
        return x, len(x), x
    try:
        mv = memoryview(x)
    except TypeError:
        b = bytes(bytearray(x))
        return b, len(b), b
    if not mv.c_contiguous:
        b = mv.tobytes()
        return b, len(b), b
    import numpy as np
    a = np.frombuffer(mv.cast('B') if mv.format != 'B' or mv.ndim != 1 else mv, dtype=np.uint8)
    if a.size == 0:
        return b'', 0, a
    return ctypes.c_char_p(a.ctypes.data), a.size, a


def _addr(arg):
    return ctypes.cast(arg if isinstance(arg, ctypes.c_char_p) else ctypes.c_char_p(arg), ctypes.c_void_p)


def _bytes(x):
    """Uint8Array / Int8Array equivalents: any buffer (bytes, bytearray, memoryview, array('b'),
    numpy int8/uint8) is taken as its raw bytes, as decode.ts:31-33 views an Int8Array."""
    if isinstance(x, (bytes, bytearray)):
        return bytes(x)
    try:
        return bytes(memoryview(x).cast('B'))
    except TypeError:
        return bytes(bytearray(x))


def brotliEncode(input, options=None):
    data, n, _keep = _in(input)
    buf = _Buf()
    rc = _L().mib_encode(data, n, ctypes.byref(_opts(options)), ctypes.byref(buf))
    if rc:
        raise _err(rc)
    return _take(buf)


class BrotliEncoder:
    """Streaming encoder: update() returns the newly completed bytes, finish() the rest."""

    def __init__(self, options=None):
        self._h = _L().mib_encoder_new(ctypes.byref(_opts(options)))
        if not self._h:
            raise BrotliError('brotli_amd: encoder creation failed')

    def update(self, chunk):
        data, n, _keep = _in(chunk)
        buf = _Buf()
        rc = _L().mib_encoder_update(self._h, data, n, ctypes.byref(buf))
        if rc:
            raise _err(rc)
        return _take(buf)

    def finish(self):
        buf = _Buf()
        rc = _L().mib_encoder_finish(self._h, ctypes.byref(buf))
        if rc:
            raise _err(rc)
        return _take(buf)

    def __del__(self):
        if getattr(self, '_h', None):
            _L().mib_encoder_free(self._h)
            self._h = None


def encoder_update_batch(encoders, chunks):
    """Advance independent BrotliEncoders by one chunk each in one GPU launch sequence;
    returns each encoder's update() result."""
    k = len(encoders)
    keep = [_in(b) for b in chunks]
    hs = (ctypes.c_void_p * k)(*[e._h for e in encoders])
    spans = (_Span * k)(*[_Span(_addr(a), n) for a, n, _ in keep])
    outs = (_Buf * k)()
    rc = _L().mib_encoder_update_batch(hs, spans, k, outs)
    if rc:
        raise _err(rc)
    return [_take(outs[i]) for i in range(k)]


def brotliDecodedSize(data):
    data, n, _keep = _in(data)
    return int(_L().mib_decoded_size(data, n))


def brotliDecode(buffer, options=None):
    """decode.ts:18-65: options = {'maxOutputSize', 'customDictionary'} or a legacy int size."""
    data, n, _keep = _in(buffer)
    exact, max_out, dic = -1, -1, None
    if isinstance(options, int) and not isinstance(options, bool):
        exact = options
    elif options:
        if options.get('maxOutputSize') is not None:
            max_out = int(options['maxOutputSize'])
        if options.get('customDictionary') is not None:
            dic = _bytes(options['customDictionary'])
    buf = _Buf()
    rc = _L().mib_decode(data, n, dic, len(dic) if dic is not None else 0, max_out, exact, ctypes.byref(buf))
    if rc == -103:   # MIB_E_OUTPUT_LIMIT: the reference's wrapper message
        raise BrotliError('Decompressed size %d exceeds limit %d' % (buf.size, max_out), rc)
    if rc:
        raise _err(rc)
    return _take(buf)


def encode_batch(buffers, options=None, gpus=None):
    """Encode independent buffers in one GPU launch sequence; returns list of bytes.  gpus:
    shard the batch over that many GPUs (0: every visible one; mib_encode_batch_n)."""
    k = len(buffers)
    keep = [_in(b) for b in buffers]
    spans = (_Span * k)(*[_Span(_addr(a), n) for a, n, _ in keep])
    outs = (_Buf * k)()
    st = (ctypes.c_int * k)()
    if gpus is None:
        rc = _L().mib_encode_batch(spans, k, ctypes.byref(_opts(options)), outs, st)
    else:
        rc = _L().mib_encode_batch_n(spans, k, ctypes.byref(_opts(options)), int(gpus), outs, st)
    if rc:
        raise _err(rc)
    res = [_take(outs[i]) for i in range(k)]
    for i in range(k):
        if st[i]:
            raise _err(st[i])
    return res


def decode_batch(buffers, gpus=None):
    """Decode independent streams on the GPU; returns a list of bytes or BrotliError.  gpus:
    shard the batch over that many GPUs (0: every visible one; mib_decode_batch_n)."""
    k = len(buffers)
    keep = [_in(b) for b in buffers]
    spans = (_Span * k)(*[_Span(_addr(a), n) for a, n, _ in keep])
    outs = (_Buf * k)()
    st = (ctypes.c_int * k)()
    if gpus is None:
        rc = _L().mib_decode_batch(spans, k, outs, st)
    else:
        rc = _L().mib_decode_batch_n(spans, k, int(gpus), outs, st)
    if rc:
        raise _err(rc)
    return [(_take(outs[i]) if st[i] == 0 else _err(st[i])) for i in range(k)]


def woff2_transform_glyf(ttf):
    """The WOFF2-transformed 'glyf' table of a TrueType font (W3C WOFF2 section 5.1), computed on
    the GPU: the FONT-mode input of brotliEncode for a WOFF2 writer (reference README.md:63)."""
    data = _bytes(ttf)
    buf = _Buf()
    rc = _L().mib_woff2_transform_glyf(data, len(data), ctypes.byref(buf))
    if rc:
        raise _err(rc)
    return _take(buf)


def woff2_transform_hmtx(ttf):
    """The WOFF2-transformed 'hmtx' table (W3C WOFF2 section 5.4), computed on the GPU, or None
    when no transform applies (both side-bearing arrays differ from the glyphs' xMin)."""
    data = _bytes(ttf)
    buf = _Buf()
    rc = _L().mib_woff2_transform_hmtx(data, len(data), ctypes.byref(buf))
    if rc:
        raise _err(rc)
    if not buf.size:
        _L().mib_buf_free(ctypes.byref(buf))
        return None
    return _take(buf)


def part_stats(ctx=None):
    """(streams decoded part-parallel, of those sent back to the serial decoder) for a
    DeviceContext, or the host API's default context"""
    a, b = ctypes.c_uint64(), ctypes.c_uint64()
    _L().mib_part_stats(ctx._c if ctx is not None else None, ctypes.byref(a), ctypes.byref(b))
    return a.value, b.value


def _prof_mode(on):
    return 2 if on == 'decode' else (1 if on else 0)


def default_profiling(on=True, clear=True):
    """Per-kernel timing (HIP events) of the host-buffer calls (brotliEncode, brotliDecode,
    BrotliEncoder, the batches): on / off / 'decode' (the decoder's kernels only), and the
    accumulated times cleared unless clear=False."""
    c = _L().mib_default_ctx()
    if not c:
        raise BrotliError('brotli_amd: no usable device')
    _L().mib_ctx_set_profiling(c, _prof_mode(on))
    if clear:
        _L().mib_ctx_clear_times(c)


def default_kernel_times():
    """{kernel: (ms, launches)} accumulated by the host-buffer calls since default_profiling()"""
    c = _L().mib_default_ctx()
    arr = (_KTime * 64)()
    n = _L().mib_ctx_kernel_times(c, arr, 64)
    return {arr[i].name.decode(): (arr[i].ms, arr[i].launches) for i in range(min(n, 64))}


class DeviceContext:
    """Device-resident batches (torch tensors / raw device pointers) for bench and the
    multi-GPU driver; wraps mib_ctx_* of include/brotli_amd.h."""

    def __init__(self, device=0, profiling=False):
        self._c = _L().mib_ctx_new(device)
        if not self._c:
            raise BrotliError('brotli_amd: no usable device %d' % device)
        _L().mib_ctx_set_profiling(self._c, _prof_mode(profiling))

    def set_profiling(self, on):
        """True / False / 'decode' (the decoder's kernels only)."""
        _L().mib_ctx_set_profiling(self._c, _prof_mode(on))

    def close(self):
        if getattr(self, '_c', None) and _lib is not None:
            _lib.mib_ctx_free(self._c)
        self._c = None

    def __del__(self):
        self.close()

    def encode(self, d_in, in_offsets, d_out, out_cap, options=None, stream=None):
        k = len(in_offsets) - 1
        ioff = (ctypes.c_uint64 * (k + 1))(*in_offsets)
        ooff = (ctypes.c_uint64 * (k + 1))()
        rc = _L().mib_ctx_encode(self._c, ctypes.byref(_opts(options)), d_in, ioff, k, d_out, out_cap, ooff, stream)
        if rc:
            raise _err(rc)
        return list(ooff)

    def decode(self, d_in, in_offsets, d_out, out_offsets, stream=None):
        k = len(in_offsets) - 1
        ioff = (ctypes.c_uint64 * (k + 1))(*in_offsets)
        ooff = (ctypes.c_uint64 * (k + 1))(*out_offsets)
        sizes = (ctypes.c_int64 * k)()
        st = (ctypes.c_int * k)()
        rc = _L().mib_ctx_decode(self._c, d_in, ioff, k, d_out, ooff, sizes, st, stream)
        if rc and rc != -104:
            raise _err(rc)
        return list(sizes), list(st)

    def kernel_times(self):
        arr = (_KTime * 32)()
        n = _L().mib_ctx_kernel_times(self._c, arr, 32)
        return {arr[i].name.decode(): (arr[i].ms, arr[i].launches) for i in range(min(n, 32))}
