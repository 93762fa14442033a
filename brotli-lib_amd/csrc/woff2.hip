// WOFF2 'glyf' transform (the FONT-mode caller of the encoder, reference
// README.md:63) on the GPU: a TrueType glyf + loca table pair becomes the seven streams of
// the W3C WOFF2 specification section 5.1 -- nContour, nPoints (255UInt16), flags,
// glyph (triplet-coded coordinate deltas + instruction lengths), composite, bbox (bitmap +
// explicit boxes) and instructions -- plus the overlap-simple bitmap.
//
// One thread per glyph, two passes: `glyf_sizes_kernel` parses each glyph (flags with
// repeats, x / y deltas, contours, components) and counts its bytes in every stream; the
// per-stream counts are scanned; `glyf_write_kernel` parses again and writes each glyph's
// bytes at its offsets.  The byte choices follow fontTools 4.62 (`WOFF2GlyfTable`), the
// implementation the tests compare against (tests/test_gpu_woff2.py).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "common.h"

namespace mib {
namespace woff2 {

enum { kNContour, kNPoints, kFlags, kGlyph, kComposite, kBBox, kInstr, kStreams };
constexpr int kHeaderBytes = 36;   // version, optionFlags, numGlyphs, indexFormat, 7 stream sizes

struct Font {                      // device view of one font's glyf / loca
  const uint8_t *glyf;
  uint32_t glyf_len;
  const uint8_t *loca;
  uint32_t num_glyphs;
  int32_t long_loca;
};

__device__ __forceinline__ uint32_t be16(const uint8_t *p) { return ((uint32_t)p[0] << 8) | p[1]; }
__device__ __forceinline__ int32_t sbe16(const uint8_t *p) { return (int16_t)be16(p); }
__device__ __forceinline__ uint32_t be32(const uint8_t *p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}
__device__ __forceinline__ int len255(uint32_t v) { return v < 253 ? 1 : v < 762 ? 2 : 3; }
__device__ __forceinline__ int put255(uint8_t *o, uint32_t v) {   // fontTools pack255UShort
  if (v < 253) {
    o[0] = (uint8_t)v;
    return 1;
  }
  if (v < 506) {
    o[0] = 255;
    o[1] = (uint8_t)(v - 253);
    return 2;
  }
  if (v < 762) {
    o[0] = 254;
    o[1] = (uint8_t)(v - 506);
    return 2;
  }
  o[0] = 253;
  o[1] = (uint8_t)(v >> 8);
  o[2] = (uint8_t)v;
  return 3;
}
// triplet encoding of one (dx, dy) (WOFF2 section 5.2): the flag byte and the data bytes
__device__ __forceinline__ int triplet(int x, int y, bool on, uint8_t *flag, uint8_t *t) {
  const int ax = x < 0 ? -x : x, ay = y < 0 ? -y : y;
  const int onb = on ? 0 : 128, xs = x < 0 ? 0 : 1, ys = y < 0 ? 0 : 1, xy = xs + 2 * ys;
  if (x == 0 && ay < 1280) {
    *flag = (uint8_t)(onb + ((ay & 0xF00) >> 7) + ys);
    t[0] = (uint8_t)ay;
    return 1;
  }
  if (y == 0 && ax < 1280) {
    *flag = (uint8_t)(onb + 10 + ((ax & 0xF00) >> 7) + xs);
    t[0] = (uint8_t)ax;
    return 1;
  }
  if (ax < 65 && ay < 65) {
    *flag = (uint8_t)(onb + 20 + ((ax - 1) & 0x30) + (((ay - 1) & 0x30) >> 2) + xy);
    t[0] = (uint8_t)((((ax - 1) & 0xF) << 4) | ((ay - 1) & 0xF));
    return 1;
  }
  if (ax < 769 && ay < 769) {
    *flag = (uint8_t)(onb + 84 + 12 * (((ax - 1) & 0x300) >> 8) + (((ay - 1) & 0x300) >> 6) + xy);
    t[0] = (uint8_t)(ax - 1);
    t[1] = (uint8_t)(ay - 1);
    return 2;
  }
  if (ax < 4096 && ay < 4096) {
    *flag = (uint8_t)(onb + 120 + xy);
    t[0] = (uint8_t)(ax >> 4);
    t[1] = (uint8_t)(((ax & 0xF) << 4) | (ay >> 8));
    t[2] = (uint8_t)ay;
    return 3;
  }
  *flag = (uint8_t)(onb + 124 + xy);
  t[0] = (uint8_t)(ax >> 8);
  t[1] = (uint8_t)ax;
  t[2] = (uint8_t)(ay >> 8);
  t[3] = (uint8_t)ay;
  return 4;
}

// TrueType glyph flags (glyf table) and component flags
constexpr int kOnCurve = 0x01, kXShort = 0x02, kYShort = 0x04, kRepeat = 0x08, kXSame = 0x10, kYSame = 0x20,
              kOverlapSimple = 0x40;
constexpr int kArgWords = 0x0001, kXYValues = 0x0002, kHaveScale = 0x0008, kMore = 0x0020, kXYScale = 0x0040,
              kTwoByTwo = 0x0080, kHaveInstr = 0x0100;
// flags a component keeps (ROUND_XY_TO_GRID, NON_OVERLAPPING, USE_MY_METRICS, OVERLAP_COMPOUND,
// SCALED / UNSCALED_COMPONENT_OFFSET); the others are recomputed
constexpr int kKeptFlags = 0x0004 | 0x0010 | 0x0200 | 0x0400 | 0x0800 | 0x1000;

// Walks one glyph; with out == nullptr only counts.  Returns false on a malformed glyph.
struct Sink {
  uint8_t *s[kStreams];   // stream cursors (write pass) or nullptr
  uint32_t n[kStreams];   // bytes per stream
  bool overlap, bbox;
};
__device__ bool walk_glyph(const Font &f, uint32_t g, Sink &k) {
  for (int i = 0; i < kStreams; i++) k.n[i] = 0;
  k.overlap = k.bbox = false;
  const uint32_t o0 = f.long_loca ? be32(f.loca + 4 * g) : 2 * be16(f.loca + 2 * g);
  const uint32_t o1 = f.long_loca ? be32(f.loca + 4 * g + 4) : 2 * be16(f.loca + 2 * g + 2);
  const bool w = k.s[0] != nullptr;
  auto emit = [&](int st, uint8_t b) {
    if (w) k.s[st][k.n[st]] = b;
    k.n[st]++;
  };
  if (o1 < o0 || o1 > f.glyf_len) return false;
  if (o1 == o0) {   // empty glyph: numberOfContours 0 and nothing else
    emit(kNContour, 0);
    emit(kNContour, 0);
    return true;
  }
  const uint8_t *p = f.glyf + o0, *end = f.glyf + o1;
  if (o1 - o0 < 10) return false;
  const int nc = sbe16(p);
  emit(kNContour, p[0]);
  emit(kNContour, p[1]);
  if (nc == 0) return true;
  const uint8_t *hdr = p;
  p += 10;
  if (nc > 0) {   // simple glyph
    if (p + 2 * nc + 2 > end) return false;
    int last = -1;
    for (int c = 0; c < nc; c++) {
      const int e = (int)be16(p + 2 * c);
      if (e <= last) return false;
      uint8_t tmp[3];
      const int m = put255(tmp, (uint32_t)(e - last));
      for (int q = 0; q < m; q++) emit(kNPoints, tmp[q]);
      last = e;
    }
    const int npts = last + 1;
    p += 2 * nc;
    const uint32_t ilen = be16(p);
    p += 2;
    const uint8_t *instr = p;
    p += ilen;
    if (p > end) return false;
    // flags (with repeats), then the x and y delta arrays they describe
    const uint8_t *fl = p;
    int nf = 0;
    const uint8_t *q = fl;
    uint32_t xbytes = 0;
    bool first = true;
    while (nf < npts) {
      if (q >= end) return false;
      const int fb = *q++;
      int rep = 1;
      if (fb & kRepeat) {
        if (q >= end) return false;
        rep += *q++;
      }
      if (first) {
        k.overlap = (fb & kOverlapSimple) != 0;
        first = false;
      }
      nf += rep;
      xbytes += (uint32_t)rep * ((fb & kXShort) ? 1u : (fb & kXSame) ? 0u : 2u);
    }
    if (nf != npts) return false;
    const uint8_t *xs = q, *ys = q + xbytes;
    // decode the points, emit flags + triplets, track the bounds
    const uint8_t *fq = fl;
    int fb = 0, rep = 0;
    int x = 0, y = 0, xmin = 0, xmax = 0, ymin = 0, ymax = 0;
    const uint8_t *xp = xs, *yp = ys;
    for (int i = 0; i < npts; i++) {
      if (rep == 0) {
        fb = *fq++;
        rep = 1;
        if (fb & kRepeat) rep += *fq++;
      }
      rep--;
      int dx, dy;
      if (fb & kXShort) {
        if (xp >= end) return false;
        dx = (fb & kXSame) ? *xp : -(int)*xp;
        xp++;
      } else if (fb & kXSame) {
        dx = 0;
      } else {
        if (xp + 2 > end) return false;
        dx = sbe16(xp);
        xp += 2;
      }
      if (fb & kYShort) {
        if (yp >= end) return false;
        dy = (fb & kYSame) ? *yp : -(int)*yp;
        yp++;
      } else if (fb & kYSame) {
        dy = 0;
      } else {
        if (yp + 2 > end) return false;
        dy = sbe16(yp);
        yp += 2;
      }
      x += dx;
      y += dy;
      if (i == 0 || x < xmin) xmin = x;
      if (i == 0 || x > xmax) xmax = x;
      if (i == 0 || y < ymin) ymin = y;
      if (i == 0 || y > ymax) ymax = y;
      uint8_t flag, t[4];
      const int m = triplet(dx, dy, (fb & kOnCurve) != 0, &flag, t);
      emit(kFlags, flag);
      for (int j = 0; j < m; j++) emit(kGlyph, t[j]);
    }
    uint8_t tmp[3];
    const int m = put255(tmp, ilen);
    for (int j = 0; j < m; j++) emit(kGlyph, tmp[j]);
    for (uint32_t j = 0; j < ilen; j++) emit(kInstr, instr[j]);
    // the explicit box only when the header's differs from the points' bounds
    const bool same = npts > 0 && sbe16(hdr + 2) == xmin && sbe16(hdr + 4) == ymin && sbe16(hdr + 6) == xmax &&
                      sbe16(hdr + 8) == ymax;
    k.bbox = !same;
  } else {   // composite glyph: the component records (re-encoded the way fontTools'
             // GlyphComponent.compile does: kept flags, minimal argument and scale forms,
             // MORE / WE_HAVE_INSTRUCTIONS recomputed), then its instructions
    bool more = true, have_instr = false;
    while (more) {
      if (p + 4 > end) return false;
      const uint32_t fl = be16(p), gid = be16(p + 2);
      const uint8_t *a = p + 4;
      int len = 4 + ((fl & kArgWords) ? 4 : 2);
      if (fl & kHaveScale) len += 2;
      else if (fl & kXYScale) len += 4;
      else if (fl & kTwoByTwo) len += 8;
      if (p + len > end) return false;
      more = (fl & kMore) != 0;
      have_instr = have_instr || (fl & kHaveInstr) != 0;
      int v0, v1;
      if (fl & kArgWords) {
        v0 = (fl & kXYValues) ? sbe16(a) : (int)be16(a);
        v1 = (fl & kXYValues) ? sbe16(a + 2) : (int)be16(a + 2);
        a += 4;
      } else {
        v0 = (fl & kXYValues) ? (int)(int8_t)a[0] : (int)a[0];
        v1 = (fl & kXYValues) ? (int)(int8_t)a[1] : (int)a[1];
        a += 2;
      }
      int t00 = 0x4000, t01 = 0, t10 = 0, t11 = 0x4000;
      const bool has_t = (fl & (kHaveScale | kXYScale | kTwoByTwo)) != 0;
      if (fl & kHaveScale) {
        t00 = t11 = sbe16(a);
      } else if (fl & kXYScale) {
        t00 = sbe16(a);
        t11 = sbe16(a + 2);
      } else if (fl & kTwoByTwo) {
        t00 = sbe16(a);
        t01 = sbe16(a + 2);
        t10 = sbe16(a + 4);
        t11 = sbe16(a + 6);
      }
      uint32_t of = (fl & kKeptFlags) | (more ? kMore : 0) | (!more && have_instr ? kHaveInstr : 0);
      bool words;
      if (fl & kXYValues) {
        of |= kXYValues;
        words = !(v0 >= -128 && v0 <= 127 && v1 >= -128 && v1 <= 127);
      } else {
        words = !(v0 >= 0 && v0 <= 255 && v1 >= 0 && v1 <= 255);
      }
      if (words) of |= kArgWords;
      int tkind = 0;   // 1 scale, 2 x and y, 3 two by two
      if (has_t) tkind = (t01 || t10) ? 3 : (t00 != t11) ? 2 : 1;
      of |= tkind == 3 ? kTwoByTwo : tkind == 2 ? kXYScale : tkind == 1 ? kHaveScale : 0;
      emit(kComposite, (uint8_t)(of >> 8));
      emit(kComposite, (uint8_t)of);
      emit(kComposite, (uint8_t)(gid >> 8));
      emit(kComposite, (uint8_t)gid);
      if (words) {
        emit(kComposite, (uint8_t)(v0 >> 8));
        emit(kComposite, (uint8_t)v0);
        emit(kComposite, (uint8_t)(v1 >> 8));
        emit(kComposite, (uint8_t)v1);
      } else {
        emit(kComposite, (uint8_t)v0);
        emit(kComposite, (uint8_t)v1);
      }
      const int tv[4] = {t00, t01, t10, t11};
      const int nt = tkind == 3 ? 4 : tkind == 2 ? 2 : tkind == 1 ? 1 : 0;
      for (int q = 0; q < nt; q++) {
        const int v = tkind == 2 ? (q == 0 ? t00 : t11) : tv[q];
        emit(kComposite, (uint8_t)(v >> 8));
        emit(kComposite, (uint8_t)v);
      }
      p += len;
    }
    if (have_instr) {
      if (p + 2 > end) return false;
      const uint32_t ilen = be16(p);
      p += 2;
      if (p + ilen > end) return false;
      uint8_t tmp[3];
      const int m = put255(tmp, ilen);
      for (int j = 0; j < m; j++) emit(kGlyph, tmp[j]);
      for (uint32_t j = 0; j < ilen; j++) emit(kInstr, p[j]);
    }
    k.bbox = true;
  }
  if (k.bbox)
    for (int j = 0; j < 8; j++) emit(kBBox, hdr[2 + j]);
  return true;
}

__global__ void glyf_sizes_kernel(Font f, uint32_t *sizes /* [kStreams][n] */, uint8_t *bits /* per glyph */,
                                  int *bad) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= f.num_glyphs) return;
  Sink k;
  for (int i = 0; i < kStreams; i++) k.s[i] = nullptr;
  if (!walk_glyph(f, g, k)) {
    atomicOr(bad, 1);
    for (int i = 0; i < kStreams; i++) k.n[i] = 0;
  }
  for (int i = 0; i < kStreams; i++) sizes[(size_t)i * f.num_glyphs + g] = k.n[i];
  bits[g] = (uint8_t)((k.overlap ? 1 : 0) | (k.bbox ? 2 : 0));
}

// offs: exclusive scans of sizes; base[s] = the stream's offset in the output
__global__ void glyf_write_kernel(Font f, const uint32_t *offs, const uint32_t *base, uint8_t *out) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= f.num_glyphs) return;
  Sink k;
  for (int i = 0; i < kStreams; i++) {
    const uint32_t extra = i == kBBox ? ((f.num_glyphs + 31) >> 5) << 2 : 0;   // the bbox bitmap comes first
    k.s[i] = out + base[i] + extra + offs[(size_t)i * f.num_glyphs + g];
  }
  walk_glyph(f, g, k);
}

// the bbox and overlap-simple bitmaps (bit 7 first), one thread per byte
__global__ void glyf_bitmaps_kernel(uint32_t n, const uint8_t *bits, uint8_t *bbox_bm, uint8_t *ovl_bm, int with_ovl) {
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t nb_bbox = ((n + 31) >> 5) << 2;
  if (b < nb_bbox) {
    uint8_t v = 0;
    for (int j = 0; j < 8; j++) {
      const uint32_t g = 8 * b + j;
      if (g < n && (bits[g] & 2)) v |= (uint8_t)(0x80 >> j);
    }
    bbox_bm[b] = v;
  }
  if (with_ovl && b < ((n + 7) >> 3)) {
    uint8_t v = 0;
    for (int j = 0; j < 8; j++) {
      const uint32_t g = 8 * b + j;
      if (g < n && (bits[g] & 1)) v |= (uint8_t)(0x80 >> j);
    }
    ovl_bm[b] = v;
  }
}


// ---------------------------------------------------------------- hmtx (WOFF2 section 5.4)
// fontTools WOFF2HmtxTable.transform: the proportional (i < numberOfHMetrics) and monospaced
// glyphs' left side bearings are dropped when every one equals its glyph's xMin (0 for an
// empty glyph).  Thread per glyph: a mismatch sets bit 0 (proportional) or 1 (monospaced).
__global__ void hmtx_check_kernel(Font f, const uint8_t *hmtx, uint32_t nhm, uint32_t *mismatch) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= f.num_glyphs) return;
  const uint32_t o0 = f.long_loca ? be32(f.loca + 4 * g) : 2 * be16(f.loca + 2 * g);
  const uint32_t o1 = f.long_loca ? be32(f.loca + 4 * g + 4) : 2 * be16(f.loca + 2 * g + 2);
  const int32_t xmin = (o1 > o0 && o0 + 10 <= f.glyf_len) ? sbe16(f.glyf + o0 + 2) : 0;
  const int32_t lsb = g < nhm ? sbe16(hmtx + 4 * g + 2) : sbe16(hmtx + 4 * nhm + 2 * (g - nhm));
  if (lsb != xmin) atomicOr(mismatch, g < nhm ? 1u : 2u);
}
// the transformed table: flags, advance widths, then the lsb array that is kept (if any)
__global__ void hmtx_write_kernel(uint32_t ng, const uint8_t *hmtx, uint32_t nhm, uint32_t keep, uint8_t *out) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= ng) return;
  if (g < nhm) {
    out[1 + 2 * g] = hmtx[4 * g];
    out[2 + 2 * g] = hmtx[4 * g + 1];
  }
  const uint32_t lsb_at = 1 + 2 * nhm;
  if (keep == 1 && g < nhm) {          // proportional glyphs' lsbs
    out[lsb_at + 2 * g] = hmtx[4 * g + 2];
    out[lsb_at + 2 * g + 1] = hmtx[4 * g + 3];
  } else if (keep == 2 && g >= nhm) {  // monospaced glyphs' lsbs
    out[lsb_at + 2 * (g - nhm)] = hmtx[4 * nhm + 2 * (g - nhm)];
    out[lsb_at + 2 * (g - nhm) + 1] = hmtx[4 * nhm + 2 * (g - nhm) + 1];
  }
}

}  // namespace woff2
}  // namespace mib

using namespace mib::woff2;

namespace {
uint32_t hbe16(const uint8_t *p) { return ((uint32_t)p[0] << 8) | p[1]; }
uint32_t hbe32(const uint8_t *p) { return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3]; }
void put16(uint8_t *p, uint32_t v) {
  p[0] = (uint8_t)(v >> 8);
  p[1] = (uint8_t)v;
}
void put32(uint8_t *p, uint32_t v) {
  p[0] = (uint8_t)(v >> 24);
  p[1] = (uint8_t)(v >> 16);
  p[2] = (uint8_t)(v >> 8);
  p[3] = (uint8_t)v;
}
}  // namespace

extern "C" int mib_ctx_ready(mib_ctx *c);
extern "C" mib_ctx *mib_default_ctx(void);
extern "C" void mib_default_lock(int on);
extern "C" void *mib_ctx_stream_of(mib_ctx *c);
extern "C" int mib_ctx_device_of(mib_ctx *c);

extern "C" int mib_woff2_transform_glyf(const uint8_t *ttf, size_t n, mib_buf *out) {
  if (!out || (!ttf && n)) return MIB_E_INVALID_ARG;
  out->data = nullptr;
  out->size = 0;
  // the sfnt table directory (host: a few dozen bytes)
  if (n < 12) return MIB_E_INVALID_ARG;
  const uint32_t ntab = hbe16(ttf + 4);
  if (12 + 16ull * ntab > n) return MIB_E_INVALID_ARG;
  uint64_t glyf_off = 0, glyf_len = 0, loca_off = 0, loca_len = 0, head_off = 0, maxp_off = 0;
  bool hg = false, hl = false, hh = false, hm = false;
  for (uint32_t i = 0; i < ntab; i++) {
    const uint8_t *r = ttf + 12 + 16 * i;
    const uint32_t off = hbe32(r + 8), len = hbe32(r + 12);
    if ((uint64_t)off + len > n) return MIB_E_INVALID_ARG;
    if (!memcmp(r, "glyf", 4)) glyf_off = off, glyf_len = len, hg = true;
    else if (!memcmp(r, "loca", 4)) loca_off = off, loca_len = len, hl = true;
    else if (!memcmp(r, "head", 4)) head_off = off, hh = true;
    else if (!memcmp(r, "maxp", 4)) maxp_off = off, hm = true;
  }
  if (!hg || !hl || !hh || !hm || head_off + 54 > n || maxp_off + 6 > n) return MIB_E_INVALID_ARG;
  const int long_loca = (int16_t)hbe16(ttf + head_off + 50) != 0 ? 1 : 0;
  const uint32_t ng = hbe16(ttf + maxp_off + 4);
  if ((uint64_t)(ng + 1) * (long_loca ? 4 : 2) > loca_len || ng == 0) return MIB_E_INVALID_ARG;
  mib_default_lock(1);
  mib_ctx *c = mib_default_ctx();
  if (!c) {
    mib_default_lock(0);
    return MIB_E_NO_DEVICE;
  }
  hipSetDevice(mib_ctx_device_of(c));
  hipStream_t st = (hipStream_t)mib_ctx_stream_of(c);
  int rc = 0;
  uint8_t *d_font = nullptr, *d_bits = nullptr, *d_out = nullptr, *d_tmp = nullptr;
  uint32_t *d_sizes = nullptr, *d_offs = nullptr, *d_base = nullptr;
  int *d_bad = nullptr;
  const size_t nsz = (size_t)kStreams * ng;
  std::vector<uint32_t> tot(kStreams);
  std::vector<uint8_t> host;
  do {
    if (hipMalloc(&d_font, glyf_len + loca_len + 16) != hipSuccess || hipMalloc(&d_sizes, 4 * nsz) != hipSuccess ||
        hipMalloc(&d_offs, 4 * nsz) != hipSuccess || hipMalloc(&d_bits, ng) != hipSuccess ||
        hipMalloc(&d_bad, 4) != hipSuccess || hipMalloc(&d_base, 4 * kStreams) != hipSuccess) {
      rc = MIB_E_OUT_OF_MEMORY;
      break;
    }
    hipMemcpyAsync(d_font, ttf + glyf_off, glyf_len, hipMemcpyHostToDevice, st);
    hipMemcpyAsync(d_font + glyf_len, ttf + loca_off, loca_len, hipMemcpyHostToDevice, st);
    hipMemsetAsync(d_bad, 0, 4, st);
    Font f{d_font, (uint32_t)glyf_len, d_font + glyf_len, ng, long_loca};
    const dim3 grid((ng + 255) / 256), block(256);
    hipLaunchKernelGGL(glyf_sizes_kernel, grid, block, 0, st, f, d_sizes, d_bits, d_bad);
    // exclusive scan of every stream's per-glyph sizes (one flat scan: each stream's run
    // starts at its own total, subtracted below)
    size_t tmp_b = 0;
    hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_b, d_sizes, d_offs, (int)nsz, st);
    if (hipMalloc(&d_tmp, tmp_b + 16) != hipSuccess) {
      rc = MIB_E_OUT_OF_MEMORY;
      break;
    }
    hipcub::DeviceScan::ExclusiveSum(d_tmp, tmp_b, d_sizes, d_offs, (int)nsz, st);
    std::vector<uint32_t> starts(kStreams + 1);
    int bad = 0;
    uint32_t last_off = 0, last_size = 0;
    for (int s = 0; s < kStreams; s++) hipMemcpyAsync(&starts[s], d_offs + (size_t)s * ng, 4, hipMemcpyDeviceToHost, st);
    hipMemcpyAsync(&last_off, d_offs + nsz - 1, 4, hipMemcpyDeviceToHost, st);
    hipMemcpyAsync(&last_size, d_sizes + nsz - 1, 4, hipMemcpyDeviceToHost, st);
    hipMemcpyAsync(&bad, d_bad, 4, hipMemcpyDeviceToHost, st);
    if (hipStreamSynchronize(st) != hipSuccess) {
      rc = MIB_E_NO_DEVICE;
      break;
    }
    if (bad) {
      rc = MIB_E_INVALID_ARG;   // a malformed glyph
      break;
    }
    starts[kStreams] = last_off + last_size;
    for (int s = 0; s < kStreams; s++) tot[s] = starts[s + 1] - starts[s];
    const uint32_t bbm = ((ng + 31) >> 5) << 2;
    tot[kBBox] += bbm;
    // output layout: header, the streams, (overlap bitmap); each stream's glyph offsets are
    // the flat scan minus the stream's start
    std::vector<uint32_t> base(kStreams);
    uint64_t pos = kHeaderBytes;
    for (int s = 0; s < kStreams; s++) {
      base[s] = (uint32_t)(pos - starts[s]);   // (unsigned wrap: base + flat offset = position)
      pos += tot[s];
    }
    // the overlap bitmap only when some simple glyph has the flag (decided after the sizes pass)
    std::vector<uint8_t> bits(ng);
    hipMemcpyAsync(bits.data(), d_bits, ng, hipMemcpyDeviceToHost, st);
    hipStreamSynchronize(st);
    bool ovl = false;
    for (uint32_t g = 0; g < ng; g++) ovl = ovl || (bits[g] & 1);
    const uint64_t total = pos + (ovl ? ((ng + 7) >> 3) : 0);
    if (hipMalloc(&d_out, total + 16) != hipSuccess) {
      rc = MIB_E_OUT_OF_MEMORY;
      break;
    }
    hipMemcpyAsync(d_base, base.data(), 4 * kStreams, hipMemcpyHostToDevice, st);
    hipLaunchKernelGGL(glyf_write_kernel, grid, block, 0, st, f, d_offs, d_base, d_out);
    const uint32_t bbox_at = (uint32_t)(base[kBBox] + starts[kBBox]);
    hipLaunchKernelGGL(glyf_bitmaps_kernel, dim3((bbm + 255) / 256), dim3(256), 0, st, ng, d_bits, d_out + bbox_at,
                       d_out + pos, ovl ? 1 : 0);
    host.resize(total);
    hipMemcpyAsync(host.data(), d_out, total, hipMemcpyDeviceToHost, st);
    if (hipStreamSynchronize(st) != hipSuccess) {
      rc = MIB_E_NO_DEVICE;
      break;
    }
    put16(&host[0], 0);
    put16(&host[2], ovl ? 1 : 0);
    put16(&host[4], ng);
    put16(&host[6], long_loca ? 1 : 0);
    for (int s = 0; s < kStreams; s++) put32(&host[8 + 4 * s], tot[s]);
    out->data = mib_buf_alloc(total);
    if (!out->data) {
      rc = MIB_E_OUT_OF_MEMORY;
      break;
    }
    memcpy(out->data, host.data(), total);
    out->size = total;
  } while (0);
  hipFree(d_font);
  hipFree(d_sizes);
  hipFree(d_offs);
  hipFree(d_bits);
  hipFree(d_bad);
  hipFree(d_base);
  hipFree(d_out);
  hipFree(d_tmp);
  mib_default_lock(0);
  return rc;
}

// WOFF2 hmtx transform (fontTools WOFF2HmtxTable.transform).  Returns 0 with out->size = 0
// when no transform applies (both side-bearing arrays must be kept: the table stays as is).
extern "C" int mib_woff2_transform_hmtx(const uint8_t *ttf, size_t n, mib_buf *out) {
  if (!out || (!ttf && n)) return MIB_E_INVALID_ARG;
  out->data = nullptr;
  out->size = 0;
  if (n < 12) return MIB_E_INVALID_ARG;
  const uint32_t ntab = hbe16(ttf + 4);
  if (12 + 16ull * ntab > n) return MIB_E_INVALID_ARG;
  uint64_t off[6] = {0, 0, 0, 0, 0, 0}, len[6] = {0, 0, 0, 0, 0, 0};
  bool have[6] = {false, false, false, false, false, false};
  static const char *kTags[6] = {"glyf", "loca", "head", "maxp", "hhea", "hmtx"};
  for (uint32_t i = 0; i < ntab; i++) {
    const uint8_t *r = ttf + 12 + 16 * i;
    const uint32_t o = hbe32(r + 8), l = hbe32(r + 12);
    if ((uint64_t)o + l > n) return MIB_E_INVALID_ARG;
    for (int t = 0; t < 6; t++)
      if (!memcmp(r, kTags[t], 4)) off[t] = o, len[t] = l, have[t] = true;
  }
  for (int t = 0; t < 6; t++)
    if (!have[t]) return MIB_E_INVALID_ARG;
  if (len[2] < 54 || len[3] < 6 || len[4] < 36) return MIB_E_INVALID_ARG;
  const int long_loca = (int16_t)hbe16(ttf + off[2] + 50) != 0 ? 1 : 0;
  const uint32_t ng = hbe16(ttf + off[3] + 4), nhm = hbe16(ttf + off[4] + 34);
  if (ng == 0 || nhm == 0 || nhm > ng || (uint64_t)(ng + 1) * (long_loca ? 4 : 2) > len[1] ||
      4ull * nhm + 2ull * (ng - nhm) > len[5])
    return MIB_E_INVALID_ARG;
  mib_default_lock(1);
  mib_ctx *c = mib_default_ctx();
  if (!c) {
    mib_default_lock(0);
    return MIB_E_NO_DEVICE;
  }
  hipSetDevice(mib_ctx_device_of(c));
  hipStream_t st = (hipStream_t)mib_ctx_stream_of(c);
  int rc = 0;
  uint8_t *d_font = nullptr, *d_out = nullptr;
  uint32_t *d_mis = nullptr;
  do {
    const uint64_t gl = len[0], ll = len[1], hl = len[5];
    if (hipMalloc(&d_font, gl + ll + hl + 16) != hipSuccess || hipMalloc(&d_mis, 4) != hipSuccess) {
      rc = MIB_E_OUT_OF_MEMORY;
      break;
    }
    hipMemcpyAsync(d_font, ttf + off[0], gl, hipMemcpyHostToDevice, st);
    hipMemcpyAsync(d_font + gl, ttf + off[1], ll, hipMemcpyHostToDevice, st);
    hipMemcpyAsync(d_font + gl + ll, ttf + off[5], hl, hipMemcpyHostToDevice, st);
    hipMemsetAsync(d_mis, 0, 4, st);
    Font f{d_font, (uint32_t)gl, d_font + gl, ng, long_loca};
    const dim3 grid((ng + 255) / 256), block(256);
    hipLaunchKernelGGL(hmtx_check_kernel, grid, block, 0, st, f, d_font + gl + ll, nhm, d_mis);
    uint32_t mis = 0;
    hipMemcpyAsync(&mis, d_mis, 4, hipMemcpyDeviceToHost, st);
    if (hipStreamSynchronize(st) != hipSuccess) {
      rc = MIB_E_NO_DEVICE;
      break;
    }
    if (mis == 3) break;   // both arrays needed: no transform
    const uint32_t keep = mis;   // 0: none, 1: proportional lsbs, 2: monospaced lsbs
    const uint64_t total = 1 + 2ull * nhm + (keep == 1 ? 2ull * nhm : keep == 2 ? 2ull * (ng - nhm) : 0);
    if (hipMalloc(&d_out, total + 16) != hipSuccess) {
      rc = MIB_E_OUT_OF_MEMORY;
      break;
    }
    hipLaunchKernelGGL(hmtx_write_kernel, grid, block, 0, st, ng, d_font + gl + ll, nhm, keep, d_out);
    out->data = mib_buf_alloc(total);
    if (!out->data) {
      rc = MIB_E_OUT_OF_MEMORY;
      break;
    }
    out->size = total;
    hipMemcpyAsync(out->data, d_out, total, hipMemcpyDeviceToHost, st);
    if (hipStreamSynchronize(st) != hipSuccess) {
      mib_buf_free(out);
      rc = MIB_E_NO_DEVICE;
      break;
    }
    out->data[0] = (uint8_t)((keep == 1 ? 0 : 1) | (keep == 2 ? 0 : 2));   // set: that array is absent
    out->size = total;
  } while (0);
  hipFree(d_font);
  hipFree(d_mis);
  hipFree(d_out);
  mib_default_lock(0);
  return rc;
}
