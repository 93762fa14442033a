"""The parse prices the distance cache (backward-references-hq.ts:309-345).

Record-structured input -- each 48-byte record repeats the one one or two records back with a
couple of bytes changed, as glyph records do -- makes the cheapest parse reuse the record
stride: after a changed byte (a literal) the copy from the same distance as the copy before it
is a last-distance copy (RFC 7932 distance code 0, implicit in command codes < 128), and a copy
from the other stride is a short code 1-15.  The parse's last-distance candidates (dp_kernel KR,
FONT mode) and the near scan's 2-3 byte copies (GENERIC / TEXT) must choose them: the oracle
decoder (the reference decoder restated) counts the distance codes of the GPU's stream, and the
stream round-trips through the oracle and the HIP decoder.
"""
import random

import pytest

import _oracle
import brotli_amd

pytestmark = pytest.mark.gpu


def records(n, seed, rec=48):
    rng = random.Random(seed)
    out = bytearray(rng.getrandbits(8) for _ in range(2 * rec))
    while len(out) < n:
        back = rec if rng.random() < 0.7 else 2 * rec
        r = bytearray(out[len(out) - back:len(out) - back + rec])
        for _ in range(rng.randrange(1, 4)):
            r[rng.randrange(rec)] = rng.getrandbits(8)
        out += r
    return bytes(out[:n])


@pytest.mark.parametrize('mode', [brotli_amd.EncoderMode.FONT, brotli_amd.EncoderMode.GENERIC])
def test_record_stride_parse_uses_the_distance_cache(mode):
    data = records(200000, 7)
    enc = brotli_amd.brotliEncode(data, {'quality': 11, 'mode': mode})
    _oracle.dist_code_counts()
    assert _oracle.decode(enc) == data
    implicit, code0, short, explicit = _oracle.dist_code_counts()
    copies = implicit + code0 + short + explicit
    print('mode %d: %d copies: implicit %d, code 0 %d, short 1-15 %d, explicit %d; %d bytes' %
          (mode, copies, implicit, code0, short, explicit, len(enc)))
    assert brotli_amd.brotliDecode(enc) == data
    # the strides come back through the cache, not as explicit distances
    assert implicit + code0 > copies // 2
    assert short > 0
    assert explicit < copies // 4
    # and the stream is far smaller than ref-fixed's on the same bytes
    ref = _oracle.encode(data[:60000], 11, 22, 2 if mode == brotli_amd.EncoderMode.FONT else 0)
    ours = brotli_amd.brotliEncode(data[:60000], {'quality': 11, 'mode': mode})
    assert len(ours) < len(ref)


def _dp_cache(on):
    import ctypes
    lib = brotli_amd._L()
    lib.mib_force_no_dp_cache.restype = None
    lib.mib_force_no_dp_cache.argtypes = [ctypes.c_int]
    lib.mib_force_no_dp_cache(0 if on else 1)


@pytest.mark.parametrize('mode', [brotli_amd.EncoderMode.GENERIC, brotli_amd.EncoderMode.TEXT, brotli_amd.EncoderMode.FONT])
def test_short_codes_come_from_the_parse(mode):
    """The parse's distance-cache candidates (dp_kernel KC: the path's ring, 15 short codes per
    node, backward-references-hq.ts:309-345) in every mode: with them the stream takes many more
    short codes 1-15 than the same parse without them (where short codes arise only when
    codes_kernel finds a chosen distance in the decoder's ring) and gets smaller."""
    data = records(200000, 11)
    try:
        _dp_cache(False)
        off = brotli_amd.brotliEncode(data, {'quality': 11, 'mode': mode})
    finally:
        _dp_cache(True)
    on = brotli_amd.brotliEncode(data, {'quality': 11, 'mode': mode})
    counts = {}
    for name, enc in (('off', off), ('on', on)):
        _oracle.dist_code_counts()
        assert _oracle.decode(enc) == data
        assert brotli_amd.brotliDecode(enc) == data
        counts[name] = _oracle.dist_code_counts()
    print('mode %d: without candidates %s, %d bytes; with %s, %d bytes' % (mode, counts['off'], len(off), counts['on'], len(on)))
    short_off, short_on = counts['off'][2], counts['on'][2]
    assert short_on > short_off + 100
    assert len(on) < len(off)


@pytest.mark.parametrize('mode', [brotli_amd.EncoderMode.GENERIC, brotli_amd.EncoderMode.FONT])
def test_candidates_parse_the_same_in_any_batch(mode):
    """A stream's parse must not depend on its batch: 24 x 1 MiB of records run the DP with two
    segments a wave (3,072 parse pieces), one of them alone with one (128 pieces); the
    candidates' pipeline (the ring history, the staircase lengths it reuses) must give the same
    bytes either way."""
    bufs = [records(1 << 20, 100 + i, rec=40 + 8 * (i % 5)) for i in range(24)]
    outs = brotli_amd.encode_batch(bufs, {'quality': 11, 'mode': mode})
    for i in (0, 7, 23):
        single = brotli_amd.brotliEncode(bufs[i], {'quality': 11, 'mode': mode})
        assert single == outs[i], i
    assert _oracle.decode(outs[7]) == bufs[7]
    assert brotli_amd.decode_batch(outs) == bufs


def test_candidates_in_every_stream_shape():
    """Binary (non-UTF-8) data takes the candidates in every encoder shape: streaming chunks
    (their candidates stay inside the chunk), part-indexed streams of >= 2 MiB (a candidate
    copy from an earlier part obeys the part lag), small windows (a candidate never reaches past
    the window), static-dictionary words and a custom dictionary on the ring (never candidate
    bases); every stream decodes with the oracle and with the HIP decoder."""
    data = records(3 << 20, 21, rec=56)
    # part-indexed one-shot stream (>= 2 MiB): HIP decodes it part-parallel
    enc = brotli_amd.brotliEncode(data, {'quality': 11})
    assert _oracle.decode(enc) == data
    assert brotli_amd.brotliDecode(enc) == data
    # streaming in 1 MiB update() chunks, and small chunks
    for step in (1 << 20, 300000):
        e = brotli_amd.BrotliEncoder({'quality': 11})
        out = b''.join([e.update(data[p:p + step]) for p in range(0, len(data), step)] + [e.finish()])
        assert brotli_amd.brotliDecode(out) == data
        assert _oracle.decode(out) == data
    small = data[:200000]
    for lg in (10, 12, 16):
        enc = brotli_amd.brotliEncode(small, {'quality': 11, 'lgwin': lg})
        assert _oracle.decode(enc) == small, lg
        assert brotli_amd.brotliDecode(enc) == small, lg
    # a custom dictionary (its tail copies push on the ring) and static-dictionary words
    cdict = records(20000, 5, rec=56)
    mixed = cdict[-3000:] + small[:100000] + b' the world of the people ' * 40
    enc = brotli_amd.brotliEncode(mixed, {'quality': 11, 'customDictionary': cdict})
    assert brotli_amd.brotliDecode(enc, {'customDictionary': cdict}) == mixed
    assert _oracle.decode(enc, dictionary=cdict) == mixed
    enc = brotli_amd.brotliEncode(mixed, {'quality': 11})
    assert _oracle.decode(enc) == mixed
    assert brotli_amd.brotliDecode(enc) == mixed
