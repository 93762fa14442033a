"""Two encode lanes (encode.hip encode_streams): a batch of >= 64 Mi positions that fits one
group runs as two halves on two HIP streams at once, lane 1 packing into a staging buffer that
is copied behind lane 0's output.  Each stream is still encoded as a call of its own: the
batch's streams equal single-stream encodes (which run one lane), and the offsets are exact
across the lane boundary (the streams either side of it decode, by HIP and by the oracle)."""
import pytest

import _oracle
import brotli_amd
from brotli_amd import datagen

pytestmark = pytest.mark.gpu


def test_two_lanes_match_single_stream_encodes():
    torch = pytest.importorskip('torch')
    # 36 streams of 1.5-2.5 MiB: ~72 MiB of positions, two lanes; unequal sizes so the halves
    # split by positions, not by count
    sizes = [(3 << 19) + (i * 37_017) % (1 << 20) for i in range(36)]
    data = datagen.enwik_device(sum(sizes), 77, torch.device('cuda', 0)).cpu().numpy().tobytes()
    bufs, o = [], 0
    for n in sizes:
        bufs.append(data[o:o + n])
        o += n
    outs = brotli_amd.encode_batch(bufs, {'quality': 11})
    dec = brotli_amd.decode_batch(outs)
    assert all(d == b for d, b in zip(dec, bufs))
    # the lane boundary lies near the middle: check the streams around it and both ends
    for i in (0, 16, 17, 18, 19, 35):
        assert outs[i] == brotli_amd.brotliEncode(bufs[i], {'quality': 11}), i
    for i in (17, 18):
        assert _oracle.decode(outs[i]) == bufs[i], i
