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
// clusters, command code, distance clusters.  Lane per metablock.
__global__ void headers_kernel(const Job *jobs, const Mb *mbs, int nmbs, const uint8_t *hdr, const uint8_t *trees,
                               uint8_t *out) {
  int m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= nmbs) return;
  const Mb &mb = mbs[m];
  const Job &jb = jobs[mb.job];
  if (jb.uncompressed) return;
  Acc a;
  a.init(reinterpret_cast<uint32_t *>(out + jb.out_off), mb.bit_off);
  for (int part = -1; part < kTreeSlots; part++) {
    const uint8_t *src = part < 0 ? hdr + (size_t)m * kHdrBytes : trees + ((size_t)m * kTreeSlots + part) * kTreeBytes;
    const uint64_t nbits = part < 0 ? mb.hdr_bits : mb.tree_bits[part];
    uint64_t i = 0;
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

// command q of its segment, with the block switches its unit places on it (same bits as
// command_bits)
template <class W>
__device__ __forceinline__ void write_command(W &wr, const Codes &cd, const Mb &mb, const uint8_t *lut, const Cmd &k,
                                              const uint8_t *lits, uint32_t p12, const Unit &u, uint32_t q) {
  if (switch_at(u, 1, q)) put_switch(wr, cd, 1, u);
  const int ct = u.type[1];
  wr.put(cd.cd[ct][k.cmd_prefix], cd.cc[ct][k.cmd_prefix]);
  const int ic = ins_code(k.ins);
  wr.put((int)kInsExtra[ic], k.ins - kInsBase[ic]);
  const uint32_t clen = k.copy ? k.copy : 2;
  const int cc = copy_code(clen);
  wr.put((int)kCopyExtra[cc], clen - kCopyBase[cc]);
  if (switch_at(u, 0, q)) put_switch(wr, cd, 0, u);
  const uint8_t *lmap = mb.lit_cmap + u.type[0] * kLitCtx;
  uint32_t p1 = p12 & 0xFF, p2 = p12 >> 8;
  for (uint32_t t = 0; t < k.ins; t++) {
    const uint32_t lit = lits[t];
    const int tree = lmap[lut[p1] | lut[256 + p2]];
    wr.put(cd.ld[tree][lit], cd.lc[tree][lit]);
    p2 = p1;
    p1 = lit;
  }
  if (k.copy && k.cmd_prefix >= 128) {
    if (switch_at(u, 2, q)) put_switch(wr, cd, 2, u);
    const uint32_t dcode = k.dist_prefix & 0x3FF;
    const int tree = mb.dist_cmap[u.type[2] * kDistCtx + dist_ctx(k.copy)];
    wr.put(cd.dd[tree][dcode], cd.dcd[tree][dcode]);
    wr.put(k.dist_prefix >> 10, k.dist_extra);
  }
}

// Block per segment: 256 commands at a time get their bit offsets from a block scan and are
// written into an LDS window, which is then stored as whole words (the chunk's first and
// last word are ORed: neighbours share them).  A command that does not fit the window (an
// insert of tens of thousands of literals) is ORed straight into global memory.
constexpr int kWinWords = 8192;   // 32 KiB = 262144 bits
__global__ __launch_bounds__(kBlock) void emit_kernel(const Job *jobs, const Seg *segs, const Mb *mbs, const Cmd *cmds,
                                                      const uint32_t *cmd_pos, const Codes *codes, const Unit *units,
                                                      uint8_t *out) {
  typedef hipcub::BlockScan<uint32_t, kBlock> Scan;
  __shared__ typename Scan::TempStorage scan_tmp;
  __shared__ uint32_t win[kWinWords];
  __shared__ uint32_t sh_fit_end;
  const Seg &sg = segs[blockIdx.x];
  const Job &jb = jobs[sg.job];
  if (jb.uncompressed) return;
  const int t = threadIdx.x;
  const Codes &cd = codes[sg.mb];
  const Mb &mb = mbs[sg.mb];
  const uint8_t *lut = kRfcContextLut + (mb.ctx_mode << 9);
  uint32_t *words = reinterpret_cast<uint32_t *>(out + jb.out_off);
  const Cmd *c = cmds + sg.cmd_off;
  const uint32_t *cp = cmd_pos + sg.cmd_off;
  const uint32_t n = sg.ncmd + (sg.extra_ins ? 1 : 0);
  const Unit *un = units + (size_t)blockIdx.x * kSubPerSeg;
  uint64_t bitpos = sg.bit_off;
  for (uint32_t base = 0; base < n; base += kBlock) {
    const uint32_t q = base + t;
    Cmd k;
    Unit u;
    uint32_t bits = 0;
    if (q < n) {
      k = c[q];
      u = un[unit_of(sg, cp[q])];
      bits = command_bits(cd, mb, lut, k, jb.data + cp[q], prev2(jb, cp[q]), u, q);
    }
    uint32_t off, total;
    Scan(scan_tmp).ExclusiveSum(bits, off, total);
    const uint32_t rel0 = (uint32_t)(bitpos & 31);
    const uint64_t w0 = bitpos >> 5;
    const uint32_t need = (uint32_t)min((uint64_t)kWinWords, ((uint64_t)rel0 + total + 31) / 32);
    for (uint32_t i = t; i < need; i += kBlock) win[i] = 0;
    if (t == 0) sh_fit_end = rel0;
    __syncthreads();
    const bool fits = (uint64_t)rel0 + off + bits <= (uint64_t)kWinWords * 32;
    if (q < n && bits) {
      if (fits) {
        OrW<false> wr;
        wr.init(win, rel0 + off);
        write_command(wr, cd, mb, lut, k, jb.data + cp[q], prev2(jb, cp[q]), u, q);
        wr.finish();
        atomicMax(&sh_fit_end, rel0 + off + bits);
      } else {
        OrW<true> wr;
        wr.init(words, bitpos + off);
        write_command(wr, cd, mb, lut, k, jb.data + cp[q], prev2(jb, cp[q]), u, q);
        wr.finish();
      }
    }
    __syncthreads();
    const uint32_t fit_end = sh_fit_end;
    const uint32_t nw = (fit_end + 31) / 32;
    for (uint32_t i = t; i < nw; i += kBlock) {
      if (i == 0 || i == nw - 1) {
        if (win[i]) atomicOr(words + w0 + i, win[i]);
      } else {
        words[w0 + i] = win[i];
      }
    }
    bitpos += total;
    __syncthreads();
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
__global__ void pack_kernel(const Job *jobs, const uint64_t *dst_off, const uint8_t *src, uint8_t *dst) {
  const Job &jb = jobs[blockIdx.y];
  uint64_t n = (jb.total_bits + 7) >> 3;
  const uint8_t *s = src + jb.out_off;
  uint8_t *d = dst + dst_off[blockIdx.y];
  for (uint64_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) d[i] = s[i];
}


void launch_emit(hipStream_t st, const Job *jobs, const Mb *mbs, int nmbs, const Seg *segs, int nsegs, const Cmd *cmds,
                 const uint32_t *cmd_pos, const Codes *codes, const Unit *units, const uint8_t *trees, const uint8_t *hdr,
                 uint8_t *out) {
  hipLaunchKernelGGL(headers_kernel, dim3((nmbs + 63) / 64), dim3(64), 0, st, jobs, mbs, nmbs, hdr, trees, out);
  hipLaunchKernelGGL(emit_kernel, dim3(nsegs), dim3(kBlock), 0, st, jobs, segs, mbs, cmds, cmd_pos, codes, units, out);
}
void launch_stored(hipStream_t st, Job *jobs, int njobs, uint8_t *out) {
  hipLaunchKernelGGL(uncompressed_kernel, dim3((unsigned)njobs), dim3(256), 0, st, jobs, njobs, out);
}
void launch_pack(hipStream_t st, const Job *jobs, int njobs, const uint64_t *dst_off, const uint8_t *src, uint8_t *dst) {
  hipLaunchKernelGGL(pack_kernel, dim3(64, (unsigned)njobs), dim3(256), 0, st, jobs, dst_off, src, dst);
}

}  // namespace enc
}  // namespace mib
