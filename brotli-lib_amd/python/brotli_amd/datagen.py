"""Deterministic synthetic inputs for the BASELINE.json workloads.

* ``xorshift32`` / ``random_bytes`` / ``ramp``: the reference's own fuzz generators
  (test/brotli.test.ts:247-260), bit-for-bit.
* ``fox``: the reference's encode bench input (bench/encode.bench.ts:7-8,14).
* ``enwik_text``: MediaWiki-XML-like text ("enwik-style"): <page> records with titles, ids,
  timestamps and a word-salad body drawn from the English word frequencies of the
  canonical corpus texts (data/words.txt), with [[links]], {{templates}}, '''bold''',
  &quot; entities and ~1/16 newlines.  Vectorised numpy; deterministic for a given
  (seed, length) on a given numpy version.
* ``glyf_stream``: WOFF2-transformed-glyf-like byte streams (see its docstring).
"""
import os

import numpy as np

_DATA = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), 'data')


def xorshift32(seed):
    """makeXorshift32 (test/brotli.test.ts:247-255)."""
    x = seed & 0xFFFFFFFF

    def nxt():
        nonlocal x
        x ^= (x << 13) & 0xFFFFFFFF
        x ^= x >> 17
        x ^= (x << 5) & 0xFFFFFFFF
        return x
    return nxt


def random_bytes(length, nxt):
    """randomBytes (test/brotli.test.ts:257-261)."""
    return bytes(nxt() & 0xFF for _ in range(length))


def ramp(length):
    return bytes(i & 0xFF for i in range(length))


def fox(repeats=1000):
    return b'The quick brown fox jumps over the lazy dog. ' * repeats


_WORDS = None


def _words():
    global _WORDS
    if _WORDS is None:
        words, counts = [], []
        with open(os.path.join(_DATA, 'words.txt'), encoding='utf-8') as f:
            for line in f:
                if line.startswith('#'):
                    continue
                w, c = line.rstrip('\n').split('\t')
                words.append(w)
                counts.append(int(c))
        p = np.asarray(counts, dtype=np.float64)
        _WORDS = (words, np.cumsum(p) / p.sum())
    return _WORDS


def _pieces_table(pieces):
    blob = b''.join(pieces)
    lens = np.fromiter((len(p) for p in pieces), dtype=np.int64, count=len(pieces))
    starts = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
    return np.frombuffer(blob, dtype=np.uint8), starts, lens


def _gather(flat, starts, lens, ids):
    ln = lens[ids]
    total = int(ln.sum())
    out_off = np.cumsum(ln) - ln
    idx = np.repeat(starts[ids] - out_off, ln) + np.arange(total, dtype=np.int64)
    return flat[idx]


def enwik_text(length, seed=1):
    """``length`` bytes of enwik-style MediaWiki XML."""
    words, cdf = _words()
    rng = np.random.default_rng(0x5EED0000 + seed)
    nw = len(words)
    caps = [w[:1].upper() + w[1:] for w in words]
    seps = [b' ', b', ', b'. ', b'.\n', b'\n', b'; ', b' (', b') ', b': ', b'\n\n']
    sep_p = np.array([0.80, 0.06, 0.05, 0.015, 0.035, 0.01, 0.008, 0.008, 0.007, 0.007])
    sep_p /= sep_p.sum()
    marks = [(b'', b''), (b'[[', b']]'), (b'{{', b'}}'), (b"'''", b"'''"), (b'&quot;', b'&quot;'), (b'[[Category:', b']]')]
    mark_p = np.array([0.925, 0.045, 0.006, 0.012, 0.008, 0.004])
    mark_p /= mark_p.sum()
    # pre-rendered page headers (titles / ids / timestamps vary per header)
    headers = []
    for h in range(512):
        t = rng.integers(0, min(nw, 3000), size=3)
        title = ' '.join(caps[i] for i in t[: 1 + h % 3])
        pid = int(rng.integers(1, 10 ** 7))
        rid = int(rng.integers(10 ** 7, 10 ** 9))
        user = caps[int(rng.integers(0, min(nw, 5000)))]
        ts = '20%02d-%02d-%02dT%02d:%02d:%02dZ' % tuple(int(v) for v in rng.integers([1, 1, 1, 0, 0, 0], [9, 13, 29, 24, 60, 60]))
        headers.append(('</text>\n    </revision>\n  </page>\n  <page>\n    <title>%s</title>\n    <ns>0</ns>\n'
                        '    <id>%d</id>\n    <revision>\n      <id>%d</id>\n      <timestamp>%s</timestamp>\n'
                        '      <contributor>\n        <username>%s</username>\n        <id>%d</id>\n'
                        '      </contributor>\n      <text xml:space="preserve">' % (
                            title, pid, rid, ts, user, pid % 99991)).encode())
    # piece ids: [0] empty, words, capitalised words, separators, mark prefixes, mark suffixes, headers
    pieces = [b''] + [w.encode() for w in words] + [c.encode() for c in caps] + seps
    pieces += [m[0] for m in marks] + [m[1] for m in marks] + headers
    W0, C0 = 1, 1 + nw
    S0 = C0 + nw
    MP0 = S0 + len(seps)
    MS0 = MP0 + len(marks)
    H0 = MS0 + len(marks)
    flat, starts, lens = _pieces_table(pieces)
    out = [b'<mediawiki xml:lang="en">\n  <page>\n    <title>Start</title>\n    <text xml:space="preserve">']
    have = len(out[0])
    while have < length:
        n = max(4096, (length - have) // 5)
        wid = np.searchsorted(cdf, rng.random(n))
        sep = rng.choice(len(seps), size=n, p=sep_p)
        # capitalise after a sentence end
        cap = np.zeros(n, dtype=bool)
        cap[1:] = (sep[:-1] == 2) | (sep[:-1] == 3) | (sep[:-1] == 9)
        word_piece = np.where(cap, C0 + wid, W0 + wid)
        mk = rng.choice(len(marks), size=n, p=mark_p)
        pre = np.where(mk > 0, MP0 + mk, 0)
        suf = np.where(mk > 0, MS0 + mk, 0)
        sep_piece = S0 + sep
        page_break = rng.random(n) < 1.0 / 900
        sep_piece = np.where(page_break, H0 + rng.integers(0, len(headers), size=n), sep_piece)
        ids = np.stack([pre, word_piece, suf, sep_piece], axis=1).reshape(-1)
        chunk = _gather(flat, starts, lens, ids).tobytes()
        out.append(chunk)
        have += len(chunk)
    return b''.join(out)[:length]


# the last bytes of every page header of enwik_device's text (below)
C5_TAIL = b'</timestamp></revision>\n    <text xml:space="preserve">'


def c5_dictionary(n=65536, seed=4999):
    """C5's custom dictionary (BASELINE.json config 5): n bytes of enwik-style text ending
    with the page-header tail the streamed text repeats."""
    return enwik_text(n - len(C5_TAIL), seed) + C5_TAIL


def c5_stream(size, seed, device):
    """C5's per-GPU input: ``size`` bytes of enwik_device text that opens with the last 120
    bytes of c5_dictionary() (host bytes)."""
    d = c5_dictionary()
    data = bytes(enwik_device(size, seed, device).cpu().numpy().tobytes())
    return d[-120:] + data[120:]


def enwik_batch(count, length, seed0):
    """``count`` independent buffers (seeds seed0 .. seed0+count-1)."""
    return [enwik_text(length, seed0 + i) for i in range(count)]


def _glyf_triplets(dx, dy, on_curve):
    """WOFF2 §5.2 triplet encoding of point deltas, vectorised: (flag stream, glyph bytes)."""
    x, y = dx.astype(np.int64), dy.astype(np.int64)
    ax, ay = np.abs(x), np.abs(y)
    sx, sy = (x >= 0).astype(np.int64), (y >= 0).astype(np.int64)
    c0 = (x == 0) & (ay < 1280)
    c1 = ~c0 & (y == 0) & (ax < 1280)
    c2 = ~c0 & ~c1 & (ax <= 64) & (ay <= 64)
    c3 = ~c0 & ~c1 & ~c2 & (ax <= 768) & (ay <= 768)
    f = np.select([c0, c1, c2, c3],
                  [((ay >> 8) << 1) + sy, 10 + ((ax >> 8) << 1) + sx,
                   20 + ((ax - 1) & 0x30) + (((ay - 1) & 0x30) >> 2) + 2 * sx + sy,
                   84 + 12 * (((ax - 1) >> 8) & 3) + ((((ay - 1) >> 8) & 3) << 2) + 2 * sx + sy],
                  120 + 2 * sx + sy)
    flags = ((f & 0x7F) | np.where(on_curve, 0, 0x80)).astype(np.uint8)
    b = np.zeros((len(x), 3), dtype=np.int64)
    b[:, 0] = np.select([c0, c1, c2, c3], [ay & 0xFF, ax & 0xFF, (((ax - 1) & 0xF) << 4) | ((ay - 1) & 0xF), (ax - 1) & 0xFF],
                        (ax >> 4) & 0xFF)
    b[:, 1] = np.where(c3, (ay - 1) & 0xFF, ((ax & 0xF) << 4) | ((ay >> 8) & 0xF))
    b[:, 2] = ay & 0xFF
    n = np.select([c0 | c1 | c2, c3], [1, 2], 3)
    keep = np.arange(3)[None, :] < n[:, None]
    return bytearray(flags.tobytes()), bytearray(b[keep].astype(np.uint8).tobytes())


def glyf_stream(length, seed=1000):
    """WOFF2 §5.1 transformed-glyf-like stream: nContour (int16 BE per glyph), nPoints
    (255UInt16 per contour), flags (1 byte / point), triplet-coded glyph coordinates,
    composite records, bbox bitmap + bbox stream and instructions, concatenated in the
    WOFF2 stream order.  Glyph shapes follow a typical text face: 1-4 contours, 4-40
    points per contour, mostly on-curve short deltas."""
    rng = np.random.default_rng(0x61F0000 + seed)
    # estimate glyph count from the target length (about 95 bytes per glyph on average)
    g = max(16, length // 95)
    ncont = rng.choice([0, 1, 2, 3, 4], size=g, p=[0.04, 0.46, 0.32, 0.13, 0.05])
    ncont_stream = ncont.astype('>i2').tobytes()
    npts = rng.integers(4, 40, size=int(ncont.sum()))
    npts_stream = bytearray()
    for v in npts:
        v = int(v)
        if v < 253:
            npts_stream.append(v)
        else:
            npts_stream += bytes([253, v >> 8, v & 0xFF])
    tot = int(npts.sum())
    on_curve = rng.random(tot) < 0.6
    dx = np.rint(rng.normal(0, 40, tot)).astype(np.int64)
    dy = np.rint(rng.normal(0, 40, tot)).astype(np.int64)
    flags, glyph = _glyf_triplets(dx, dy, on_curve)
    # instruction lengths (255UInt16 per simple glyph) go to the glyph stream, bodies to instructions
    simple = int((ncont > 0).sum())
    ilen = rng.integers(0, 60, size=simple)
    for v in ilen:
        glyph.append(int(v))
    instr = rng.integers(0, 256, size=int(ilen.sum()), dtype=np.uint8)
    instr[::3] = rng.choice([0x40, 0x41, 0x1D, 0x1E, 0x2B, 0x5D, 0xB0, 0xB8], size=instr[::3].shape)
    comp = int((ncont == 0).sum())
    composite = bytearray()
    for _ in range(comp):
        composite += bytes([0x00, 0x23, 0, int(rng.integers(0, 255)), int(rng.integers(0, 64)), int(rng.integers(0, 64)),
                            0x00, 0x22, 0, int(rng.integers(0, 255)), 0, 0])
    bbox_bitmap = bytes(((g + 31) >> 5) << 2)
    bbox = rng.integers(-200, 1800, size=4 * max(1, g // 20)).astype('>i2').tobytes()
    out = ncont_stream + bytes(npts_stream) + bytes(flags) + bytes(glyph) + bytes(composite) + bbox_bitmap + bbox + instr.tobytes()
    if len(out) < length:
        out = (out * (length // max(1, len(out)) + 1))
    return out[:length]


def enwik_device(total, seed, device):
    """``total`` bytes of enwik-style text generated directly in device memory (torch).

    Same piece tables and distributions as ``enwik_text`` (so the same statistics), drawn
    with a seeded torch generator on the device: one GiB takes well under a second, where
    the numpy path needs ~100 s.  Deterministic for (total, seed) on a given torch build;
    it is bench input only -- parity fixtures use ``enwik_text``.
    """
    import torch
    words, cdf = _words()
    rng = np.random.default_rng(0x5EED0000 + seed)
    nw = len(words)
    caps = [w[:1].upper() + w[1:] for w in words]
    seps = [b' ', b', ', b'. ', b'.\n', b'\n', b'; ', b' (', b') ', b': ', b'\n\n']
    sep_p = np.array([0.80, 0.06, 0.05, 0.015, 0.035, 0.01, 0.008, 0.008, 0.007, 0.007])
    marks = [(b'', b''), (b'[[', b']]'), (b'{{', b'}}'), (b"'''", b"'''"), (b'&quot;', b'&quot;'), (b'[[Category:', b']]')]
    mark_p = np.array([0.925, 0.045, 0.006, 0.012, 0.008, 0.004])
    headers = []
    for h in range(512):
        t = rng.integers(0, min(nw, 3000), size=3)
        title = ' '.join(caps[i] for i in t[: 1 + h % 3])
        pid = int(rng.integers(1, 10 ** 7))
        headers.append(('</text>\n  </page>\n  <page>\n    <title>%s</title>\n    <id>%d</id>\n'
                        '    <revision><id>%d</id><timestamp>20%02d-%02d-%02dT12:00:00Z</timestamp></revision>\n'
                        '    <text xml:space="preserve">' % (title, pid, pid * 7 + 13, h % 9 + 1, h % 12 + 1,
                                                              h % 28 + 1)).encode())
    pieces = [b''] + [w.encode() for w in words] + [c.encode() for c in caps] + seps
    pieces += [m[0] for m in marks] + [m[1] for m in marks] + headers
    W0, C0 = 1, 1 + nw
    S0 = C0 + nw
    MP0 = S0 + len(seps)
    MS0 = MP0 + len(marks)
    H0 = MS0 + len(marks)
    flat, starts, lens = _pieces_table(pieces)
    dev = torch.device(device)
    flat_t = torch.from_numpy(flat.copy()).to(dev)
    starts_t = torch.from_numpy(starts).to(dev)
    lens_t = torch.from_numpy(lens).to(dev)
    cdf_t = torch.from_numpy(cdf).to(dev)
    sep_pt = torch.from_numpy(sep_p / sep_p.sum()).to(dev)
    mark_pt = torch.from_numpy(mark_p / mark_p.sum()).to(dev)
    g = torch.Generator(device=dev)
    g.manual_seed(0x5EED0000 + seed)
    out = torch.empty(total, dtype=torch.uint8, device=dev)
    have = 0
    while have < total:
        n = int(min(max(4096, (total - have) // 5), 1 << 23))
        wid = torch.searchsorted(cdf_t, torch.rand(n, generator=g, device=dev, dtype=torch.float64)).clamp_(max=nw - 1)
        sep = torch.multinomial(sep_pt, n, replacement=True, generator=g)
        cap = torch.zeros(n, dtype=torch.bool, device=dev)
        cap[1:] = (sep[:-1] == 2) | (sep[:-1] == 3) | (sep[:-1] == 9)
        word_piece = torch.where(cap, C0 + wid, W0 + wid)
        mk = torch.multinomial(mark_pt, n, replacement=True, generator=g)
        pre = torch.where(mk > 0, MP0 + mk, torch.zeros_like(mk))
        suf = torch.where(mk > 0, MS0 + mk, torch.zeros_like(mk))
        sep_piece = S0 + sep
        brk = torch.rand(n, generator=g, device=dev) < 1.0 / 900
        hdr = H0 + torch.randint(0, len(headers), (n,), generator=g, device=dev)
        sep_piece = torch.where(brk, hdr, sep_piece)
        ids = torch.stack([pre, word_piece, suf, sep_piece], dim=1).reshape(-1)
        ln = lens_t[ids]
        csum = torch.cumsum(ln, 0)
        tot = int(csum[-1])
        take = min(tot, total - have)
        base = torch.repeat_interleave(starts_t[ids] - (csum - ln), ln, output_size=tot)
        idx = base + torch.arange(tot, device=dev)
        out[have:have + take] = flat_t[idx[:take]]
        have += take
    return out
