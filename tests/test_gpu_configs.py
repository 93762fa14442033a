"""BASELINE.json's single-GPU configurations as parity tests, through the C ABI.

C2: one 64 MiB (67,108,864 B) enwik-style buffer, q11 GENERIC lgwin 22, encoded on the GPU
    and decoded by the HIP decoder AND by the oracle (the reference decoder restated), both
    bit-exact at the full size; plus the reference-encoded (oracle) stream of a golden-sized
    prefix decoded on the GPU.
C3: 1024 x 262,144 B WOFF2-transformed glyf tables (glyph sets from the reference's Inter
    font, jittered per seed 1000+i; datagen.glyf_font_batch), q11 FONT, through
    encode_batch and the device-resident context; every stream decoded by the HIP decoder,
    a sample by the oracle.
C4: the per-GPU shard, 1024 x 1 MiB enwik-style buffers, q11: every stream HIP-decoded, 16 by
    the oracle.  (C5 at full size: tests/test_gpu_custom_dict.py.)
Plus: a context on the last visible device round-trips (per-device decoder tables).
"""
import pytest

import _oracle
import brotli_amd
from brotli_amd import datagen

pytestmark = pytest.mark.gpu
MIB = 1 << 20


def test_c2_single_64mib_stream_q11():
    d = datagen.enwik_text(64 * MIB, 2)
    assert len(d) == 67108864
    enc = brotli_amd.brotliEncode(d, {'quality': 11, 'lgwin': 22})
    assert len(enc) < len(d) // 2
    got = _oracle.decode(enc)
    assert isinstance(got, bytes) and got == d, 'oracle decode of the GPU stream'
    assert brotli_amd.brotliDecode(enc) == d, 'HIP decode of the GPU stream'
    # 64 MiB is four 16 MiB metablocks (encode.ts:206), so the reference's header peek
    # (engine.ts:2155-2192: the first metablock must be the last) has no size for it either
    assert brotli_amd.brotliDecodedSize(enc) == -1 == _oracle.peek_size(enc)
    # the reference's own encoder (oracle, ref-fixed) on a prefix: decoded on the GPU
    ref = _oracle.encode(d[:300000], 11, 22)
    assert brotli_amd.brotliDecode(ref) == d[:300000]


def test_c3_glyf_batch_font_mode():
    k, n = 1024, 262144
    bufs = datagen.glyf_font_batch(k, n, 1000, workers=8)
    outs = brotli_amd.encode_batch(bufs, {'quality': 11, 'mode': brotli_amd.EncoderMode.FONT})
    dec = brotli_amd.decode_batch(outs)
    bad = [i for i in range(k) if dec[i] != bufs[i]]
    assert not bad, bad[:10]
    for i in range(0, k, 97):   # the oracle on a sample
        assert _oracle.decode(outs[i]) == bufs[i], i
    ratio = sum(map(len, outs)) / (k * n)
    ref = sum(len(_oracle.encode(bufs[i], 11, 22, 2)) for i in range(0, 8))
    ours = sum(len(outs[i]) for i in range(0, 8))
    print('C3 ratio %.4f; first 8: GPU %d vs ref-fixed %d bytes (%.4f)' % (ratio, ours, ref, ours / ref))
    assert ours < 0.92 * ref   # (measured 0.83: the FONT-mode 4-byte keys and last-distance copies)


def test_c4_per_gpu_shard_1024x1mib_q11():
    """C4's per-GPU shard at full size, exactly as bench.py runs it on rank 0: 1024 x 1 MiB
    enwik-style buffers (enwik_device, seed 2000) encoded q11 lgwin 22 through the
    device-resident context; the HIP decoder returns every buffer bit-exactly, and the oracle
    (the reference decoder restated) decodes 16 of the GPU streams to the same bytes."""
    torch = pytest.importorskip('torch')
    k, n = 1024, MIB
    dev = torch.device('cuda', 0)
    data = datagen.enwik_device(k * n, 2000, dev)
    cap = k * n + k * n // 8 + 4096 * k
    comp = torch.empty(cap, dtype=torch.uint8, device=dev)
    ctx = brotli_amd.DeviceContext(0)
    off = ctx.encode(data.data_ptr(), [i * n for i in range(k + 1)], comp.data_ptr(), cap, {'quality': 11, 'lgwin': 22})
    slot = n + 4096
    out = torch.empty(k * slot, dtype=torch.uint8, device=dev)
    sizes, status = ctx.decode(comp.data_ptr(), off, out.data_ptr(), [i * slot for i in range(k + 1)])
    assert status == [0] * k and sizes == [n] * k
    assert torch.equal(out.view(k, slot)[:, :n], data.view(k, n))
    raw = comp[:off[-1]].cpu().numpy().tobytes()
    host = data.cpu().numpy().tobytes()
    for i in range(0, k, 64):
        assert _oracle.decode(raw[off[i]:off[i + 1]]) == host[i * n:(i + 1) * n], i
    ratio = off[-1] / (k * n)
    print('C4 shard ratio %.5f' % ratio)
    assert ratio < 0.40


def test_c3_device_context_matches_batch():
    torch = pytest.importorskip('torch')
    k, n = 64, 262144
    bufs = datagen.glyf_font_batch(k, n, 1000, workers=8)
    opts = {'quality': 11, 'mode': 2}
    host = brotli_amd.encode_batch(bufs, opts)
    dev = torch.device('cuda', 0)
    data = torch.frombuffer(bytearray(b''.join(bufs)), dtype=torch.uint8).to(dev)
    cap = k * (n + n // 8 + 4096)
    comp = torch.empty(cap, dtype=torch.uint8, device=dev)
    ctx = brotli_amd.DeviceContext(0)
    off = ctx.encode(data.data_ptr(), [i * n for i in range(k + 1)], comp.data_ptr(), cap, opts)
    raw = comp[:off[-1]].cpu().numpy().tobytes()
    assert [raw[off[i]:off[i + 1]] for i in range(k)] == host
    slot = n + 4096
    out = torch.empty(k * slot, dtype=torch.uint8, device=dev)
    sizes, status = ctx.decode(comp.data_ptr(), off, out.data_ptr(), [i * slot for i in range(k + 1)])
    assert status == [0] * k and sizes == [n] * k
    assert torch.equal(out.view(k, slot)[:, :n], data.view(k, n))


def test_context_on_last_device():
    torch = pytest.importorskip('torch')
    last = torch.cuda.device_count() - 1
    d = datagen.enwik_text(300000, 5)
    dev = torch.device('cuda', last)
    data = torch.frombuffer(bytearray(d), dtype=torch.uint8).to(dev)
    cap = len(d) + 8192
    comp = torch.empty(cap, dtype=torch.uint8, device=dev)
    ctx = brotli_amd.DeviceContext(last)
    off = ctx.encode(data.data_ptr(), [0, len(d)], comp.data_ptr(), cap, {'quality': 11})
    out = torch.empty(len(d) + 4096, dtype=torch.uint8, device=dev)
    sizes, status = ctx.decode(comp.data_ptr(), off, out.data_ptr(), [0, len(d) + 4096])
    assert status == [0] and sizes == [len(d)]
    assert bytes(out[:len(d)].cpu().numpy().tobytes()) == d
    assert _oracle.decode(comp[:off[1]].cpu().numpy().tobytes()) == d


def test_default_context_from_threads():
    """ctypes drops the GIL: concurrent brotliEncode / brotliDecode on the default context
    are serialised by the library (runtime.cpp g_default_mu), never interleaved."""
    from concurrent.futures import ThreadPoolExecutor
    bufs = [datagen.enwik_text(200000 + 4099 * i, 40 + i) for i in range(8)]

    def trip(d):
        enc = brotli_amd.brotliEncode(d, {'quality': 11 if len(d) % 2 else 9})
        return enc, brotli_amd.brotliDecode(enc)

    with ThreadPoolExecutor(8) as ex:
        res = list(ex.map(trip, bufs * 2))
    for (enc, dec), d in zip(res, bufs * 2):
        assert dec == d
        assert _oracle.decode(enc) == d
