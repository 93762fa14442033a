"""Batches sharded over GPUs inside the C ABI (mib_encode_batch_n / mib_decode_batch_n,
brotli-lib_amd/csrc/multi.cpp; SURVEY.md §8(b),(e)).  Shard s runs on device s % device count,
so on a one-GPU box two shards share device 0 and these tests exercise the real sharding
(forced by mib_force_shards: by default one device runs the one-context calls):
size-balanced assignment, one host thread and context per shard, results back in input
order.  The 8-GPU node itself is the driver's; here the streams must equal the one-GPU
batch byte for byte (each stream's encoding depends on its own bytes only) and decode to
the inputs on the HIP decoder and the oracle."""
import ctypes

import pytest

import _oracle
import brotli_amd
from brotli_amd import datagen

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _shard_path():
    # one device runs the sharded calls as the one-context batch; the tests force the shard
    # machinery (threads, contexts, assignment) onto it
    lib = brotli_amd._L()
    lib.mib_force_shards.restype = None
    lib.mib_force_shards.argtypes = [ctypes.c_int]
    lib.mib_force_shards(1)
    yield
    lib.mib_force_shards(0)


def _mixed():
    # sizes span the framings: empty, < 64 B (stored), small, ~1 MiB, and > 2 MiB (part index)
    bufs = [b'', b'abc', datagen.enwik_text(100, 1), datagen.glyf_stream(70000, 1001)]
    bufs += [datagen.enwik_text(20000 + 7919 * i, 50 + i) for i in range(20)]
    bufs += [datagen.enwik_text(1 << 20, 90), datagen.enwik_text(3 << 20, 91)]
    return bufs


@pytest.mark.parametrize('gpus', [2, 3, 0])
def test_sharded_encode_equals_single(gpus):
    bufs = _mixed()
    one = brotli_amd.encode_batch(bufs, {'quality': 11})
    many = brotli_amd.encode_batch(bufs, {'quality': 11}, gpus=gpus)
    assert many == one
    dec = brotli_amd.decode_batch(many, gpus=gpus)
    assert dec == bufs
    for i in (3, 10, len(bufs) - 1):
        assert _oracle.decode(many[i]) == bufs[i]


def test_single_device_runs_the_one_context_call():
    lib = brotli_amd._L()
    lib.mib_force_shards(0)
    bufs = _mixed()[:12]
    one = brotli_amd.encode_batch(bufs, {'quality': 11})
    assert brotli_amd.encode_batch(bufs, {'quality': 11}, gpus=4) == one
    assert brotli_amd.decode_batch(one, gpus=4) == bufs


def test_sharded_decode_errors_stay_in_their_slots():
    bufs = _mixed()[:10]
    enc = brotli_amd.encode_batch(bufs, {'quality': 9}, gpus=2)
    bad = bytes([0x1b, 0x3f, 0xff, 0xff])
    got = brotli_amd.decode_batch(enc[:5] + [bad] + enc[5:], gpus=2)
    assert got[:5] == bufs[:5] and got[6:] == bufs[5:]
    assert isinstance(got[5], brotli_amd.BrotliError)
    want = _oracle.decode(bad)
    assert got[5].code == want
