"""A small, fast pin for the decoder's literal path.

Mid-round 3 a working build decoded some of the 1024 C3 streams (FONT mode, context-modelled
literals) to wrong bytes; only the full-size C3 batch caught it.  The change being made then
rewrote the literal loop of fast_loop: the literal byte placed in its output lane by
`v_writelane` (through m0, which the same loop's LDS-DMA also uses for its LDS address) and
one branch around the second-level table lookup.  This test drives exactly that path in about
a second: skewed bytes over all 256 values (literal codes longer than 8 bits, so the
second-level tables are read), a different distribution after each class of previous byte
(SIGNED / UTF8 contexts split them into several literal codes), literal runs of 1-200 bytes
that cross 64-byte output lines, and runs of short copies (near: overlapping; far) between
them -- copy -> literal (the literal context waits for the copy's bytes) and copy -> copy
(several source loads in flight) transitions.  Encoded on the GPU (FONT and GENERIC), decoded
by the HIP decoder in one batch and by the oracle on a sample; plus the oracle's own (ref-fixed)
streams of the same data decoded on the GPU.
"""
import functools

import numpy as np
import pytest

import _oracle
import brotli_amd

pytestmark = pytest.mark.gpu


def lit_stress(n, seed):
    rng = np.random.default_rng(seed)
    # per class of the previous byte (p1 >> 6), a Zipf-like law over a permutation whose most
    # likely values lie in the next class: the contexts predict very different bytes
    draws = []   # per class: pre-drawn bytes of its law, taken in order
    for k in range(4):
        nxt = (k + 1) & 3
        own = rng.permutation(np.arange(64 * nxt, 64 * nxt + 64))
        rest = rng.permutation(np.setdiff1d(np.arange(256), own))
        perm = np.concatenate([own, rest])
        w = 1.0 / np.arange(1, 257) ** (0.8 + 0.15 * k)
        cdf = np.cumsum(w / w.sum())
        draws.append(perm[np.minimum(255, np.searchsorted(cdf, rng.random(n)))].tolist())
    at = [0, 0, 0, 0]
    out = bytearray()
    prev = 0
    while len(out) < n:
        run = int(rng.integers(1, 200))
        for _ in range(run):
            k = prev >> 6
            prev = draws[k][at[k]]
            at[k] += 1
            out.append(prev)
        if len(out) > 64:
            for _ in range(int(rng.integers(0, 5))):   # a run of copies
                ln = int(rng.integers(4, 48))
                d = int(rng.integers(1, 64)) if rng.random() < 0.3 else int(rng.integers(64, len(out)))
                d = min(d, len(out))
                for _ in range(ln):
                    out.append(out[len(out) - d])
                prev = out[-1]
    return bytes(out[:n])


@functools.lru_cache(maxsize=1)
def _bufs():
    return [lit_stress(65536 + 4099 * i, 500 + i) for i in range(32)]


@pytest.mark.parametrize('mode', [brotli_amd.EncoderMode.FONT, brotli_amd.EncoderMode.GENERIC])
def test_context_modelled_literals_second_level_tables(mode):
    bufs = _bufs()
    outs = brotli_amd.encode_batch(bufs, {'quality': 11, 'mode': mode})
    dec = brotli_amd.decode_batch(outs)
    bad = [i for i in range(len(bufs)) if dec[i] != bufs[i]]
    assert not bad, bad[:10]
    for i in range(0, len(bufs), 8):
        assert _oracle.decode(outs[i]) == bufs[i], i
        assert brotli_amd.brotliDecode(outs[i]) == bufs[i], i   # one stream per call: the BIG build
    # the reference's own (ref-fixed) encoder on the same data
    refs = [_oracle.encode(bufs[i], 11, 22, int(mode)) for i in range(0, 8)]
    assert brotli_amd.decode_batch(refs) == bufs[:8]
