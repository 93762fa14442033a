"""Encoder-side customDictionary (mib_enc_opts.dict) and BASELINE config C5.

The reference encoder has no dictionary option (src/encode/encode.ts:22-27); its decoder takes a
`customDictionary` and resolves a copy whose distance exceeds the window's maximum as a
compound-dictionary copy (src/decode/engine.ts:142-159,903-1011).  That decoder accepts only a
copy ending exactly at the dictionary's last byte (engine.ts:992; tests/golden/decode_compound.json
pins it), so the encoder only ever emits those: a copy of the dictionary's last L bytes, distance
min(pos, max distance) + L.  What must hold:
  * the stream decodes to the input with the same dictionary, on the oracle (the reference
    decoder restated) and on the HIP decoder -- one-shot, batch and streaming;
  * dictionary copies are really emitted where the input repeats the dictionary's tail and the
    window has nothing (the oracle counts them), and they shrink the stream;
  * C5 at its full size: one 1 GiB stream through BrotliEncoder.update() in 1 MiB chunks, q9,
    lgwin 24, with a dictionary; decoded by the oracle and by the HIP decoder.
"""
import pytest

import _oracle
import brotli_amd
from brotli_amd import datagen

pytestmark = pytest.mark.gpu

c5_dictionary = datagen.c5_dictionary


def _both(data, stream, d):
    got = _oracle.decode(stream, dictionary=d)
    assert isinstance(got, bytes) and got == data, 'oracle decode with the dictionary'
    assert brotli_amd.brotliDecode(stream, {'customDictionary': d}) == data, 'HIP decode with the dictionary'


@pytest.mark.parametrize('q,lgwin', [(11, 22), (9, 24), (5, 18), (10, 16)])
def test_one_shot_tail_copies(q, lgwin):
    d = c5_dictionary()
    # the dictionary's tail where the window has nothing to offer: the stream start, and the
    # first occurrences of its shorter suffixes later on
    data = d[-180:] + datagen.enwik_text(120000, 3) + d[-97:-40] + d[-40:] + datagen.enwik_text(50000, 4)
    r0 = _oracle.compound_refs()
    enc = brotli_amd.brotliEncode(data, {'quality': q, 'lgwin': lgwin, 'customDictionary': d})
    _both(data, enc, d)
    assert _oracle.compound_refs() > r0, 'no dictionary copy was emitted'
    plain = brotli_amd.brotliEncode(data, {'quality': q, 'lgwin': lgwin})
    if q >= 10 and lgwin <= 22:
        # static-dictionary words are in play here, and the decoder addresses them past the
        # custom dictionary (engine.ts:907): every word costs more distance bits, so the
        # dictionary's tail copies may not pay for that on this input
        assert len(enc) < 1.005 * len(plain), (len(enc), len(plain))
    else:
        assert len(enc) < len(plain), (len(enc), len(plain))
    # the stream needs its dictionary: without it the reference decoder fails or differs
    alone = _oracle.decode(enc)
    assert alone != data


@pytest.mark.parametrize('q', [11, 9])
def test_tail_copy_ending_on_a_parse_piece_boundary(q):
    """a dictionary tail copy that ends exactly on an 8 KiB parse-piece
    boundary B has distance min(B - L, max) + L = B; a window copy starting at B that repeats
    the stream's first bytes has distance B too.  Joining the two (as two window copies of one
    distance are joined across pieces) would make one dictionary copy longer than the tail:
    the reference decoder reads past the dictionary and fails.  Each piece boundary of the
    first segment is tried, with unique bytes around it."""
    import random
    d = c5_dictionary(8192, 21)
    rnd = random.Random(99)
    for B in (8192, 16384, 40960):
        L = 37
        head = bytes(rnd.getrandbits(8) for _ in range(B - L))
        data = head + d[-L:] + head[:300] + bytes(rnd.getrandbits(8) for _ in range(5000))
        r0 = _oracle.compound_refs()
        enc = brotli_amd.brotliEncode(data, {'quality': q, 'customDictionary': d})
        _both(data, enc, d)
        assert _oracle.compound_refs() > r0, 'the tail copy before the boundary was not emitted'


def test_int8_dictionary_and_small_inputs():
    import array
    d = c5_dictionary(4096, 7)
    d8 = array.array('b', d)   # Int8Array view of the same bytes
    for data in (d[-64:], d[-70:] + b'x' * 10, d[-4:] + b'tail', b'', b'abc', d[-300:]):
        enc = brotli_amd.brotliEncode(data, {'customDictionary': d8})
        _both(data, enc, d)
    # a dictionary too short to copy from is accepted and changes nothing
    data = datagen.enwik_text(50000, 8)
    assert brotli_amd.brotliEncode(data, {'customDictionary': b'ab'}) == brotli_amd.brotliEncode(data)


def test_batch_and_device_context():
    d = c5_dictionary(20000, 11)
    bufs = [d[-(50 + 13 * i):] + datagen.enwik_text(30000 + 997 * i, 20 + i) for i in range(12)]
    opts = {'quality': 11, 'customDictionary': d}
    outs = brotli_amd.encode_batch(bufs, opts)
    for b, o in zip(bufs, outs):
        _both(b, o, d)
        assert o == brotli_amd.brotliEncode(b, opts)   # a batch encodes each stream as alone


def test_streaming_with_dictionary():
    d = c5_dictionary()
    data = d[-150:] + datagen.enwik_text(10 << 20, 31)
    r0 = _oracle.compound_refs()
    e = brotli_amd.BrotliEncoder({'quality': 9, 'lgwin': 24, 'mode': 1, 'customDictionary': d,
                                  'streamChunk': 4 << 20})   # several device chunks
    stream = b''.join([e.update(data[i:i + (1 << 20)]) for i in range(0, len(data), 1 << 20)] + [e.finish()])
    _both(data, stream, d)
    assert _oracle.compound_refs() > r0


def test_c5_one_gib_stream_q9_lgwin24_dictionary():
    """BASELINE config C5 per GPU at its full size: 1 GiB of enwik-style TEXT through
    BrotliEncoder.update() in 1 MiB chunks, q9, lgwin 24, custom dictionary; the stream is
    decoded by the oracle and by the HIP decoder (part-parallel, with the dictionary)."""
    torch = pytest.importorskip('torch')
    size = 1 << 30
    d = c5_dictionary()
    data = datagen.c5_stream(size, 5000, torch.device('cuda', 0))   # opens with the dictionary's tail
    e = brotli_amd.BrotliEncoder({'quality': 9, 'lgwin': 24, 'mode': 1, 'customDictionary': d})
    step = 1 << 20
    parts = []
    for i in range(0, size, step):
        parts.append(e.update(data[i:i + step]))
    parts.append(e.finish())
    stream = b''.join(parts)
    del parts
    print('C5 1 GiB with dictionary: %d bytes (%.4f)' % (len(stream), len(stream) / size))
    assert len(stream) < size // 2
    p0, f0 = brotli_amd.part_stats()
    got = brotli_amd.brotliDecode(stream, {'customDictionary': d})
    assert got == data, 'HIP decode'
    assert brotli_amd.part_stats() == (p0 + 1, f0), 'the 1 GiB stream was not decoded part-parallel'
    del got
    r0 = _oracle.compound_refs()
    got = _oracle.decode(stream, dictionary=d)
    assert isinstance(got, bytes) and got == data, 'oracle decode'
    assert _oracle.compound_refs() > r0
