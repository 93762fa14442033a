// Bit emission: metablock headers and prefix codes, the
// commands of each segment at their final bit offsets, stored (uncompressed) framing, and the
// packing of finished streams.
#include <hipcub/hipcub.hpp>

#include "enc_common.h"

namespace mib {
namespace enc {

// lane-private bit accumulator for the metablock headers; edge words are atomicOr'ed
struct Acc {   // lane-private bit accumulator writing 32-bit words; edge words are atomicOr'ed
  uint32_t *base;
  uint64_t pos;      // absolute bit position of the next bit
  uint64_t acc;      // pending bits
  int nacc;
  uint64_t first_word;
  __device__ void init(uint32_t *b, uint64_t p) {
    base = b;
    pos = p;
    acc = 0;
    nacc = (int)(p & 31);
    first_word = p >> 5;
  }
  __device__ void flush_word(bool last) {
    uint64_t wi = (pos - nacc) >> 5;
    uint32_t v = (uint32_t)acc;
    if (wi == first_word || last) atomicOr(base + wi, v);
    else base[wi] = v;
    acc >>= 32;
    nacc -= 32;
  }
  __device__ void put(int n, uint64_t v) {   // n <= 32
    if (!n) return;
    acc |= (v & ((1ull << n) - 1)) << nacc;
    nacc += n;
    pos += n;
    if (nacc >= 32) flush_word(false);
  }
  __device__ void finish() {
    if (nacc > 0) {
      uint64_t wi = (pos - nacc) >> 5;
      atomicOr(base + wi, (uint32_t)acc);
    }
  }
};


// metablock header (with its context maps) + its prefix codes in stream order: literal
// clusters, command code, distance clusters.  Wave per metablock: part 0 is the header, part
// k + 1 tree slot k; lane l copies the parts [l P, (l + 1) P) to their bit offsets (a wave
// scan of the part sizes), its own contiguous range of the output (edge words atomicOr'ed).
// (One lane per metablock copied ~3 KiB bit by bit: 0.2 ms for a single metablock, r05m.)
constexpr int kHdrParts = kTreeSlots + 1;
constexpr int kHdrPer = (kHdrParts + 63) / 64;
__global__ __launch_bounds__(64) void headers_kernel(const Job *jobs, const Mb *mbs, int nmbs, const uint8_t *hdr,
                                                     const uint8_t *trees, uint8_t *out) {
  const int m = blockIdx.x, lane = threadIdx.x;
  if (m >= nmbs) return;
  const Mb &mb = mbs[m];
  const Job &jb = jobs[mb.job];
  if (jb.uncompressed) return;
  auto bits_of = [&](int part) -> uint64_t { return part >= kHdrParts ? 0u : part == 0 ? mb.hdr_bits : mb.tree_bits[part - 1]; };
  uint64_t mine = 0;
#pragma unroll
  for (int q = 0; q < kHdrPer; q++) mine += bits_of(lane * kHdrPer + q);
  uint64_t incl = mine;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint64_t y = __shfl_up(incl, o);
    if (lane >= o) incl += y;
  }
  if (!mine) return;
  Acc a;
  a.init(reinterpret_cast<uint32_t *>(out + jb.out_off), mb.bit_off + incl - mine);
  for (int q = 0; q < kHdrPer; q++) {
    const int part = lane * kHdrPer + q;
    const uint64_t nbits = bits_of(part);
    if (!nbits) continue;
    const uint8_t *src = part == 0 ? hdr + (size_t)m * kHdrBytes : trees + ((size_t)m * kTreeSlots + part - 1) * kTreeBytes;
    uint64_t i = 0;
    for (; i + 32 <= nbits; i += 32)
      a.put(32, (uint32_t)src[i >> 3] | ((uint32_t)src[(i >> 3) + 1] << 8) | ((uint32_t)src[(i >> 3) + 2] << 16) |
                    ((uint32_t)src[(i >> 3) + 3] << 24));
    for (; i + 8 <= nbits; i += 8) a.put(8, src[i >> 3]);
    if (i < nbits) a.put((int)(nbits - i), src[i >> 3]);
  }
  a.finish();
}

// Bit accumulator that ORs whole 32-bit words into a word array (LDS window or global).
template <bool kGlobal>
struct OrW {
  uint32_t *w;
  uint32_t wi;
  uint64_t acc;
  int nacc;
  __device__ void init(uint32_t *base, uint64_t bitpos) {
    w = base;
    wi = (uint32_t)(bitpos >> 5);
    nacc = (int)(bitpos & 31);
    acc = 0;
  }
  __device__ void put(int n, uint32_t v) {   // n <= 32
    if (!n) return;
    acc |= (uint64_t)(v & (uint32_t)((1ull << n) - 1)) << nacc;
    nacc += n;
    if (nacc >= 32) {
      atomicOr(w + wi, (uint32_t)acc);
      wi++;
      acc >>= 32;
      nacc -= 32;
    }
  }
  __device__ void finish() {
    if (nacc > 0) atomicOr(w + wi, (uint32_t)acc);
  }
};

// a block switch: block type code, block count code, count extra bits (storeBlockSwitch,
// metablock.ts:204-220)
template <class W>
__device__ __forceinline__ void put_switch(W &wr, const Codes &cd, int cat, const Unit &u) {
  const int code = u.sw_code[cat], bc = block_count_code(u.sw_count[cat]);
  wr.put(cd.btd[cat][code], cd.btc[cat][code]);
  wr.put(cd.bcd[cat][bc], cd.bcc[cat][bc]);
  wr.put((int)kBlkBits[bc], u.sw_count[cat] - kBlkOff[bc]);
}

// item k of command q (see item_bits in enc_common.h: same bits, in stream order)
template <class W>
__device__ __forceinline__ void write_item(W &wr, const Codes &cd, const Mb &mb, const uint16_t *cmap, const uint8_t *lut, const Job &jb,
                                           const Cmd &c, uint32_t p, const Seg &sg, const Unit *su, uint32_t q, uint32_t k) {
  const Unit &u = su[unit_of(sg, p)];
  if (k == 0) {
    if (switch_at(u, 1, q)) put_switch(wr, cd, 1, u);
    const int ct = u.type[1];
    wr.put(cd.cd[ct][c.cmd_prefix], cd.cc[ct][c.cmd_prefix]);
    const int ic = ins_code(c.ins);
    wr.put((int)kInsExtra[ic], c.ins - kInsBase[ic]);
    const uint32_t clen = c.copy ? c.copy : 2;
    const int cc = copy_code(clen);
    wr.put((int)kCopyExtra[cc], clen - kCopyBase[cc]);
  } else if (k <= c.ins) {
    const uint32_t lp = p + k - 1;
    const Unit &ul = su[unit_of(sg, lp)];
    if (lit_switch_at(ul, lp)) put_switch(wr, cd, 0, ul);
    const uint32_t lit = jb.data[lp];
    const int tree = literal_tree(cmap, lut, ul, prev2(jb, lp));
    wr.put(cd.ld[tree][lit], cd.lc[tree][lit]);
  } else if (c.copy && c.cmd_prefix >= 128) {
    if (switch_at(u, 2, q)) put_switch(wr, cd, 2, u);
    const uint32_t dcode = c.dist_prefix & 0x3FF;
    const int tree = mb.dist_cmap[u.type[2] * kDistCtx + dist_ctx(c.copy)];
    wr.put(cd.dd[tree][dcode], cd.dcd[tree][dcode]);
    wr.put(c.dist_prefix >> 10, c.dist_extra);
  }
}

// Item k of command q when it carries no block switch (the common case): its bits and its
// whole bit string (<= 15 + 24 + 24 bits), so the write pass ORs it without looking the codes up
// again; an item with a switch returns false and is written by write_item.
__device__ __forceinline__ bool item_packed(const Codes &cd, const Mb &mb, const uint16_t *cmap, const uint8_t *lut, const Job &jb,
                                            const Cmd &c, uint32_t p, const Seg &sg, const Unit *su, uint32_t q, uint32_t k,
                                            uint32_t &bits, uint64_t &val) {
  const Unit &u = su[unit_of(sg, p)];
  if (k == 0) {
    if (switch_at(u, 1, q)) return false;
    const int ct = u.type[1];
    const int ic = ins_code(c.ins);
    const uint32_t clen = c.copy ? c.copy : 2;
    const int cc = copy_code(clen);
    const uint32_t n0 = cd.cd[ct][c.cmd_prefix], n1 = kInsExtra[ic], n2 = kCopyExtra[cc];
    val = (uint64_t)cd.cc[ct][c.cmd_prefix] | ((uint64_t)(c.ins - kInsBase[ic]) << n0) | ((uint64_t)(clen - kCopyBase[cc]) << (n0 + n1));
    bits = n0 + n1 + n2;
    return true;
  }
  if (k <= c.ins) {
    const uint32_t lp = p + k - 1;
    const Unit &ul = su[unit_of(sg, lp)];
    if (lit_switch_at(ul, lp)) return false;
    const uint32_t lit = jb.data[lp];
    const int tree = literal_tree(cmap, lut, ul, prev2(jb, lp));
    bits = cd.ld[tree][lit];
    val = cd.lc[tree][lit];
    return true;
  }
  if (!c.copy || c.cmd_prefix < 128) {
    bits = 0;
    val = 0;
    return true;
  }
  if (switch_at(u, 2, q)) return false;
  const uint32_t dcode = c.dist_prefix & 0x3FF;
  const int tree = mb.dist_cmap[u.type[2] * kDistCtx + dist_ctx(c.copy)];
  const uint32_t n0 = cd.dd[tree][dcode];
  val = (uint64_t)cd.dcd[tree][dcode] | ((uint64_t)c.dist_extra << n0);
  bits = n0 + (c.dist_prefix >> 10);
  return true;
}

// Blocks per segment: block (s, y) writes segment s's tiles of kEmitTile commands y, y +
// gridDim.y, ...; a tile starts at the segment's bit offset plus its earlier tiles' bits
// (sizes_kernel's tile_bits), so a call of few segments (a streaming chunk: 16) still spreads
// its commands over many blocks.  A tile's commands are taken kBlock at a time and expanded
// into their items (header, literals, distance); kEmitItems items per lane per pass get their
// bit offsets from a block scan and are ORed into an LDS window, which is then stored as whole
// words (the pass's first and last word are ORed: neighbours share them).  A pass is at most
// kBlock * kEmitItems items of <= 180 bits, so it always fits the window.
constexpr int kWinWords = 8192;   // 32 KiB = 262144 bits
constexpr int kEmitItems = 4;
static_assert(kBlock * kEmitItems * 180 <= kWinWords * 32 - 64, "emit tile must fit the LDS window");
__global__ __launch_bounds__(kBlock) void emit_kernel(const Job *jobs, const Seg *segs, const Mb *mbs, const Cmd *cmds,
                                                      const uint32_t *cmd_pos, const Codes *codes, const Unit *units,
                                                      const uint32_t *tile_bits, uint8_t *out) {
  static_assert(kEmitTile % kBlock == 0, "a tile is whole command blocks");
  typedef hipcub::BlockScan<uint32_t, kBlock> Scan;
  __shared__ typename Scan::TempStorage scan_tmp;
  __shared__ uint32_t win[kWinWords];
  __shared__ ItemMap<kBlock> map;
  __shared__ Cmd sh_c[kBlock];
  __shared__ uint32_t sh_p[kBlock];
  __shared__ Unit sh_u[kSubPerSeg];
  __shared__ uint32_t sh_tile[kEmitTiles];   // the tiles' bit offsets within the segment
  const Seg &sg = segs[blockIdx.x];
  const Job &jb = jobs[sg.job];
  if (jb.uncompressed) return;
  const uint32_t n = sg.ncmd + (sg.extra_ins ? 1 : 0);
  const uint32_t ntile = (n + kEmitTile - 1) / kEmitTile;
  if (blockIdx.y >= ntile) return;
  const int t = threadIdx.x;
  if (t < 64) {   // exclusive prefix sum of the tile sizes (at most 65), a wave step of 64
    const uint32_t *tb = tile_bits + (size_t)blockIdx.x * kEmitTiles;
    uint32_t carry = 0;
    for (uint32_t q0 = 0; q0 < ntile; q0 += 64) {
      const uint32_t q = q0 + t, v = q < ntile ? tb[q] : 0;
      uint32_t inc = v;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(inc, o);
        if (t >= o) inc += y;
      }
      if (q < ntile) sh_tile[q] = carry + inc - v;
      carry += __shfl(inc, 63);
    }
  }
  const Codes &cd = codes[sg.mb];
  const Mb &mb = mbs[sg.mb];
  __shared__ uint8_t sh_lut[512];   // per-literal lookups from LDS
  __shared__ uint16_t sh_cmap[kLitSlots];
  for (int i = t; i < 512; i += kBlock) sh_lut[i] = kRfcContextLut[(mb.ctx_mode << 9) + i];
  for (int i = t; i < kLitSlots; i += kBlock) sh_cmap[i] = mb.lit_cmap[i];
  __syncthreads();
  const uint8_t *lut = sh_lut;
  uint32_t *words = reinterpret_cast<uint32_t *>(out + jb.out_off);
  const Cmd *c = cmds + sg.cmd_off;
  const uint32_t *cp = cmd_pos + sg.cmd_off;
  if (t < kSubPerSeg) sh_u[t] = units[(size_t)blockIdx.x * kSubPerSeg + t];
  __syncthreads();
  for (uint32_t tile = blockIdx.y; tile < ntile; tile += gridDim.y) {
  uint64_t bitpos = sg.bit_off + sh_tile[tile];
  const uint32_t tend = min(n, (tile + 1) * kEmitTile);
  for (uint32_t base = tile * kEmitTile; base < tend; base += kBlock) {
    const uint32_t nb = min((uint32_t)kBlock, tend - base);
    uint32_t cnt = 0;
    if ((uint32_t)t < nb) {
      sh_c[t] = c[base + t];
      sh_p[t] = cp[base + t];
      cnt = item_count(sh_c[t]);
    }
    uint32_t off, nitems;
    Scan(scan_tmp).ExclusiveSum(cnt, off, nitems);
    map.off[t] = off;
    if (t == 0) map.off[nb] = nitems;   // (nb <= kBlock; a later slot j > nb is never read)
    __syncthreads();
    for (uint32_t i0 = 0; i0 < nitems; i0 += kBlock * kEmitItems) {
      uint32_t bits[kEmitItems], qj[kEmitItems], kk[kEmitItems];
      uint64_t val[kEmitItems];
      uint32_t packed = 0;   // bit e: item e was packed (a bit mask: a bool array indexed by the
                             // loop counter lived in scratch memory, a store and four loads per item)
      const uint32_t first = i0 + (uint32_t)t * kEmitItems;
      uint32_t j = first < nitems ? map.find(first, nb) : 0;
      for (int e = 0; e < kEmitItems; e++) {
        const uint32_t i = first + e;
        bits[e] = 0;
        qj[e] = j;
        kk[e] = 0;
        val[e] = 0;
        packed |= 1u << e;
        if (i < nitems) {
          while (map.off[j + 1] <= i) j++;
          qj[e] = j;
          kk[e] = i - map.off[j];
          const Cmd &k = sh_c[j];
          const uint32_t p = sh_p[j];
          if (!item_packed(cd, mb, sh_cmap, lut, jb, k, p, sg, sh_u, base + j, kk[e], bits[e], val[e])) {
            packed &= ~(1u << e);
            bits[e] = item_bits(cd, mb, sh_cmap, lut, jb, k, p, sg, sh_u, base + j, kk[e]);
          }
        }
      }
      uint32_t boff[kEmitItems], total;
      Scan(scan_tmp).ExclusiveSum(bits, boff, total);
      const uint32_t rel0 = (uint32_t)(bitpos & 31);
      const uint64_t w0 = bitpos >> 5;
      const uint32_t nw = (rel0 + total + 31) / 32;
      for (uint32_t w = t; w < nw; w += kBlock) win[w] = 0;
      __syncthreads();
      for (int e = 0; e < kEmitItems; e++) {
        if (!bits[e]) continue;
        if (packed >> e & 1) {   // the whole item: at most 63 bits over three words
          const uint32_t b = rel0 + boff[e], w = b >> 5, sh = b & 31;
          const uint64_t lo = val[e] << sh;
          atomicOr(win + w, (uint32_t)lo);
          if (bits[e] + sh > 32) atomicOr(win + w + 1, (uint32_t)(lo >> 32));
          if (bits[e] + sh > 64) atomicOr(win + w + 2, (uint32_t)(val[e] >> (64 - sh)));
          continue;
        }
        const uint32_t jj = qj[e];
        const Cmd &k = sh_c[jj];
        const uint32_t p = sh_p[jj];
        OrW<false> wr;
        wr.init(win, rel0 + boff[e]);
        write_item(wr, cd, mb, sh_cmap, lut, jb, k, p, sg, sh_u, base + jj, kk[e]);
        wr.finish();
      }
      __syncthreads();
      for (uint32_t w = t; w < nw; w += kBlock) {
        if (w == 0 || w == nw - 1) {
          if (win[w]) atomicOr(words + w0 + w, win[w]);
        } else {
          words[w0 + w] = win[w];
        }
      }
      bitpos += total;
      __syncthreads();
    }
  }
  }
}

// quality 0 / n < 64 (encode.ts:105-138, storeUncompressedMetaBlock metablock.ts:821-850), the
// empty stream (:92-103), and streams whose compressed form came out larger: window bits,
// stored metablocks of up to 2^24 - 1 bytes, then ISLAST+ISEMPTY on the final chunk.
__global__ void uncompressed_kernel(Job *jobs, int njobs, uint8_t *out) {
  Job &jb = jobs[blockIdx.x];
  if (!jb.uncompressed) return;
  uint8_t *o = out + jb.out_off;
  __shared__ uint64_t hpos;
  const uint32_t maxb = (1u << 24) - 1;
  uint64_t bitpos = 0;
  if (jb.uncompressed == 2) {
    // a fallback stream may hold partial compressed bits: clear what the stored form covers
    uint64_t clear = min((uint64_t)jb.n + 5ull * ((jb.n >> 24) + 1) + 8, jb.out_cap);
    for (uint64_t q = threadIdx.x; q < clear; q += blockDim.x) o[q] = 0;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    BitW w{o, 0};
    if (jb.hdr_lgwin) put_window_bits(w, (int)jb.hdr_lgwin);
    hpos = w.pos;
  }
  __syncthreads();
  bitpos = hpos;
  for (uint32_t pos = 0; pos < jb.n;) {
    uint32_t bs = min(jb.n - pos, maxb);
    __syncthreads();
    if (threadIdx.x == 0) {
      BitW w{o, bitpos};
      w.put(1, 0);
      int l2 = bs == 1 ? 1 : 32 - __clz(bs - 1);
      int mn = (l2 < 16 ? 16 : l2 + 3) / 4;
      w.put(2, (uint32_t)(mn - 4));
      w.put(mn * 4, bs - 1);
      w.put(1, 1);
      hpos = (w.pos + 7) & ~7ull;
    }
    __syncthreads();
    uint64_t byte0 = hpos >> 3;
    for (uint32_t k = threadIdx.x; k < bs; k += blockDim.x) o[byte0 + k] = jb.data[pos + k];
    bitpos = (byte0 + bs) * 8;
    pos += bs;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    if (jb.final_) {
      BitW w{o, bitpos};
      w.put(1, 1);
      w.put(1, 1);
      bitpos = (w.pos + 7) & ~7ull;
    }
    jb.total_bits = bitpos;
  }
}

// pack the per-job output slices back to back
// Each stream's place in the packed output (dst_off[0..k]: out_pos, then its sizes summed) and
// the call's status in dst_off[k + 1]: 0, or a stream's bytes past its scratch slot / the packed
// output past out_cap (then nothing is packed).  One block; the host reads it all back with
// the jobs after the pack (it used to read the jobs, sum on the host and upload the offsets
// before the pack: a host round trip per call, ~50 us of a cadence update()).
__global__ __launch_bounds__(1024) void dst_off_kernel(const Job *jobs, int k, uint64_t out_pos, uint64_t out_cap,
                                                        uint64_t *dst_off) {
  typedef hipcub::BlockScan<uint64_t, 1024> Scan;
  __shared__ typename Scan::TempStorage tmp;
  __shared__ int bad;
  const int t = threadIdx.x, per = (k + 1023) / 1024, lo = min(k, t * per), hi = min(k, lo + per);
  if (t == 0) bad = 0;
  __syncthreads();
  uint64_t sum = 0;
  for (int j = lo; j < hi; j++) {
    const uint64_t nb = (jobs[j].total_bits + 7) >> 3;
    if (nb > jobs[j].out_cap) atomicOr(&bad, 1);
    sum += nb;
  }
  uint64_t x, total;
  Scan(tmp).ExclusiveSum(sum, x, total);
  x += out_pos;
  for (int j = lo; j < hi; j++) {
    dst_off[j] = x;
    x += (jobs[j].total_bits + 7) >> 3;
  }
  __syncthreads();
  if (t == 0) {
    dst_off[k] = out_pos + total;
    dst_off[k + 1] = bad ? (uint64_t)1 : (out_pos + total > out_cap ? (uint64_t)2 : (uint64_t)0);
  }
}
__global__ void pack_kernel(const Job *jobs, const uint64_t *dst_off, int k, const uint8_t *src, uint8_t *dst) {
  if (dst_off[k + 1]) return;   // (dst_off_kernel's status: nothing to pack)
  const Job &jb = jobs[blockIdx.y];
  uint64_t n = (jb.total_bits + 7) >> 3;
  const uint8_t *s = src + jb.out_off;
  uint8_t *d = dst + dst_off[blockIdx.y];
  for (uint64_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) d[i] = s[i];
}


void launch_emit(hipStream_t st, const Job *jobs, const Mb *mbs, int nmbs, const Seg *segs, int nsegs, const Cmd *cmds,
                 const uint32_t *cmd_pos, const Codes *codes, const Unit *units, const uint32_t *tile_bits,
                 const uint8_t *trees, const uint8_t *hdr, uint8_t *out) {
  if (nmbs) hipLaunchKernelGGL(headers_kernel, dim3(nmbs), dim3(64), 0, st, jobs, mbs, nmbs, hdr, trees, out);
  // blocks per segment: enough for ~2,048 blocks (a batch of >= 2,048 segments: one, each
  // looping over its tiles); blocks past a segment's last tile return at once
  static const int target = knob("MIB_EMIT_BLOCKS") ? std::max(1, atoi(knob("MIB_EMIT_BLOCKS"))) : 2048;   // (experiments)
  const int per = std::min(kEmitTiles, std::max(1, (target + nsegs - 1) / std::max(nsegs, 1)));
  hipLaunchKernelGGL(emit_kernel, dim3(nsegs, per), dim3(kBlock), 0, st, jobs, segs, mbs, cmds, cmd_pos, codes, units,
                     tile_bits, out);
}
void launch_stored(hipStream_t st, Job *jobs, int njobs, uint8_t *out) {
  hipLaunchKernelGGL(uncompressed_kernel, dim3((unsigned)njobs), dim3(256), 0, st, jobs, njobs, out);
}
void launch_pack(hipStream_t st, const Job *jobs, int njobs, uint64_t out_pos, uint64_t out_cap, uint64_t *dst_off,
                 const uint8_t *src, uint8_t *dst) {
  hipLaunchKernelGGL(dst_off_kernel, dim3(1), dim3(1024), 0, st, jobs, njobs, out_pos, out_cap, dst_off);
  hipLaunchKernelGGL(pack_kernel, dim3(64, (unsigned)njobs), dim3(256), 0, st, jobs, dst_off, njobs, src, dst);
}

}  // namespace enc
}  // namespace mib
