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


# ---------------------------------------------------------------------------- C3 from a real font
# C3's buffers are WOFF2-transformed glyf tables whose parameters come from the
# reference's Inter bench font (bench/fixtures/enc-ttf.bin, kept in tests/golden/bench), perturbed
# per seed.  glyf_font(seed) builds a TrueType glyph set from the font's glyphs -- drawn at random
# with replacement, each simple glyph's points jittered by a few font units -- and
# glyf_font_stream() runs the WOFF2 glyf transform on it (the GPU's, woff2_transform_glyf: the
# FONT-mode producer of §8 f4) and cuts the transformed table to the buffer size.
_FONT = None
_BENCH = os.path.join(os.path.dirname(os.path.dirname(_DATA)), 'tests', 'golden', 'bench')


def _sfnt_tables(font):
    import struct
    n = struct.unpack('>H', font[4:6])[0]
    out = {}
    for i in range(n):
        tag, _, off, ln = struct.unpack('>4sIII', font[12 + 16 * i:28 + 16 * i])
        out[tag.decode('latin-1')] = font[off:off + ln]
    return out


def _font_glyphs():
    """the bench font's glyphs: ('s', contour ends, instructions, on-curve flags, xs, ys) per
    simple glyph, ('c', raw bytes) per composite one, None for an empty one"""
    global _FONT
    if _FONT is not None:
        return _FONT
    import struct
    with open(os.path.join(_BENCH, 'enc-ttf.bin'), 'rb') as f:
        font = f.read()
    t = _sfnt_tables(font)
    long_loca = struct.unpack('>h', t['head'][50:52])[0] == 1
    ng = struct.unpack('>H', t['maxp'][4:6])[0]
    loca = (struct.unpack('>%dI' % (ng + 1), t['loca'][:4 * (ng + 1)]) if long_loca else
            tuple(2 * v for v in struct.unpack('>%dH' % (ng + 1), t['loca'][:2 * (ng + 1)])))
    glyf = t['glyf']
    gl = []
    for g in range(ng):
        b = glyf[loca[g]:loca[g + 1]]
        if not b:
            gl.append(None)
            continue
        nc = struct.unpack('>h', b[:2])[0]
        if nc < 0:
            gl.append(('c', bytes(b)))
            continue
        raw = bytes(b)
        ends = struct.unpack('>%dH' % nc, b[10:10 + 2 * nc])
        p = 10 + 2 * nc
        il = struct.unpack('>H', b[p:p + 2])[0]
        instr = bytes(b[p + 2:p + 2 + il])
        p += 2 + il
        npts = ends[-1] + 1 if nc else 0
        flags = []
        while len(flags) < npts:
            f = b[p]
            p += 1
            flags.append(f)
            if f & 8:
                flags += [f] * b[p]
                p += 1
        coords = []
        for short, same in ((2, 16), (4, 32)):
            v, vals = 0, []
            for f in flags:
                if f & short:
                    d = b[p]
                    p += 1
                    v += d if f & same else -d
                elif not f & same:
                    v += struct.unpack('>h', b[p:p + 2])[0]
                    p += 2
                vals.append(v)
            coords.append(vals)
        gl.append(('s', ends, instr, [f & 1 for f in flags], coords[0], coords[1], raw))
    _FONT = gl
    return gl


def _encode_simple(ends, instr, on, xs, ys):
    """a TrueType simple glyph (flags with repeats, short / same coordinates, bbox recomputed)"""
    import struct
    flags, xb, yb = [], bytearray(), bytearray()
    px = py = 0
    for o, x, y in zip(on, xs, ys):
        f = o
        for d, short, same, buf in ((x - px, 2, 16, xb), (y - py, 4, 32, yb)):
            if d == 0:
                f |= same
            elif -256 < d < 256:
                f |= short | (same if d > 0 else 0)
                buf.append(abs(d))
            else:
                buf += struct.pack('>h', d)
        flags.append(f)
        px, py = x, y
    fb = bytearray()
    i = 0
    while i < len(flags):
        r = 1
        while i + r < len(flags) and flags[i + r] == flags[i] and r < 256:
            r += 1
        if r > 1:
            fb += bytes([flags[i] | 8, r - 1])
        else:
            fb.append(flags[i])
        i += r
    hdr = struct.pack('>hhhhh', len(ends), min(xs), min(ys), max(xs), max(ys))
    return hdr + struct.pack('>%dH' % len(ends), *ends) + struct.pack('>H', len(instr)) + instr + bytes(fb) + bytes(xb) + bytes(yb)


def _remap_composite(b, ng, rng):
    """a composite glyph whose components point at glyphs of the new set"""
    import struct
    b = bytearray(b)
    p = 10
    while True:
        fl = struct.unpack('>H', b[p:p + 2])[0]
        b[p + 2:p + 4] = struct.pack('>H', int(rng.integers(0, ng)))
        p += 4 + (4 if fl & 1 else 2)
        p += 2 if fl & 8 else 4 if fl & 0x40 else 8 if fl & 0x80 else 0
        if not fl & 0x20:
            return bytes(b)


def glyf_font(seed, nglyphs=3000, jitter=0.35):
    """a TrueType font (head, maxp, loca, glyf) of `nglyphs` glyphs drawn from the bench font
    with replacement; a `jitter` share of the simple glyphs get 30 % of their points moved by
    up to 3 font units (seed-determined), the others are the font's own bytes"""
    import struct
    src = _font_glyphs()
    rng = np.random.default_rng(0x6F00000 + seed)
    out = []
    for g in rng.integers(0, len(src), size=nglyphs):
        s = src[int(g)]
        if s is None:
            out.append(b'')
        elif s[0] == 'c':
            out.append(_remap_composite(s[1], nglyphs, rng))
        elif rng.random() >= jitter:
            out.append(s[6])
        else:
            _, ends, instr, on, xs, ys, _ = s
            n = len(xs)
            j = rng.random(n) < 0.3
            dx = np.where(j, rng.integers(-3, 4, size=n), 0)
            dy = np.where(j, rng.integers(-3, 4, size=n), 0)
            out.append(_encode_simple(ends, instr, on, [int(v) for v in np.asarray(xs) + dx], [int(v) for v in np.asarray(ys) + dy]))
    out = [g + b'\0' * (-len(g) & 3) for g in out]   # 4-byte aligned glyphs
    loca = [0]
    for g in out:
        loca.append(loca[-1] + len(g))
    tabs = _sfnt_tables(open(os.path.join(_BENCH, 'enc-ttf.bin'), 'rb').read())
    head = bytearray(tabs['head'])
    head[50:52] = struct.pack('>h', 1)   # long loca
    maxp = bytearray(tabs['maxp'])
    maxp[4:6] = struct.pack('>H', nglyphs)
    tables = {'glyf': b''.join(out), 'head': bytes(head), 'loca': struct.pack('>%dI' % len(loca), *loca), 'maxp': bytes(maxp)}
    tags = sorted(tables)
    off = 12 + 16 * len(tags)
    dirs, body = b'', b''
    for t in tags:
        data = tables[t]
        dirs += struct.pack('>4sIII', t.encode(), 0, off + len(body), len(data))
        body += data + b'\0' * (-len(data) & 3)
    return struct.pack('>IHHHH', 0x00010000, len(tags), 64, 2, 0) + dirs + body


def glyf_font_stream(length, seed, transform=None):
    """C3's buffer: the WOFF2-transformed glyf table of glyf_font(seed), cut to `length` bytes
    (transform: the glyf transform to use; default the GPU's)"""
    if transform is None:
        from brotli_amd import woff2_transform_glyf as transform
    n = 5600
    while True:
        t = transform(glyf_font(seed, n))
        if len(t) >= length:
            return t[:length]
        n = int(n * (length / max(1, len(t))) * 1.1) + 64


def _font_job(a):
    seed, n = a
    return glyf_font(seed, n)


def glyf_font_batch(count, length, seed0, workers=8, transform=None):
    """C3's batch: glyf_font_stream(length, seed0 + i) for i < count; the fonts are built on
    `workers` processes, the transforms run here (on the GPU by default)"""
    from concurrent.futures import ProcessPoolExecutor
    if transform is None:
        from brotli_amd import woff2_transform_glyf as transform
    seeds = [seed0 + i for i in range(count)]
    with ProcessPoolExecutor(max(1, workers)) as ex:
        fonts = list(ex.map(_font_job, [(s, 5600) for s in seeds], chunksize=8))
    out = []
    for s, f in zip(seeds, fonts):
        t = transform(f)
        out.append(t[:length] if len(t) >= length else glyf_font_stream(length, s, transform))
    return out
