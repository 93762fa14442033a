// Entropy coding: commands -> prefix codes, per-metablock
// histograms, length-limited Huffman codes and their serialisation, bit sizes / offsets.
//
// Every stage here is parallel over segments (a block each) or over (metablock, alphabet);
// the only per-stream serial steps (carry, offsets, dist_ring) touch O(segments) values.
#include <hipcub/hipcub.hpp>
#include <cstdlib>
#include <algorithm>

#include "enc_common.h"

namespace mib {
namespace enc {

// ---------------------------------------------------------------- carry: lane per stream
// Literals left after a segment's last copy belong to the next command, which may be in a
// later segment; a metablock's final literals form an insert-only command (createInsertCommand
// path of encode.ts:240-262).  Also the decoder's last distance at each segment start: the
// distance ring's slot 0 always holds the previous copy's distance (a code-0 command does not
// push, but reuses exactly that distance), so code 0 is decidable per segment in parallel.
//
// Wave per stream, 64 segments per step: both are prefix scans over the metablock's segments
// (carry: a segment with copies resets it to its trailing literals, one without adds them; last
// distance: a segment with copies sets it).
__global__ __launch_bounds__(64) void carry_kernel(Job *jobs, int njobs, Seg *segs, const Mb *mbs) {
  const int j = blockIdx.x, lane = threadIdx.x;
  if (j >= njobs) return;
  Job &jb = jobs[j];
  if (jb.uncompressed) return;
  uint32_t pd = (uint32_t)jb.dc_in[0];
  for (uint32_t m = 0; m < jb.nmb; m++) {
    const Mb &mb = mbs[jb.mb_base + m];
    uint32_t carry = 0;
    const uint32_t end = mb.first_seg + mb.nseg;
    for (uint32_t c0 = mb.first_seg; c0 < end; c0 += 64) {
      const uint32_t s = c0 + lane;
      const bool live = s < end;
      uint32_t ncmd = 0, tail = 0, last = 0;
      if (live) {
        ncmd = segs[s].ncmd;
        tail = segs[s].tail_lits;
        last = segs[s].last_dist;
      }
      // (reset?, value) summaries, composed by an inclusive wave scan
      uint32_t cr = ncmd ? 1u : 0u, cv = tail, pr = cr, pv = last;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t ycr = (uint32_t)__shfl_up((int)cr, o), ycv = (uint32_t)__shfl_up((int)cv, o);
        const uint32_t ypr = (uint32_t)__shfl_up((int)pr, o), ypv = (uint32_t)__shfl_up((int)pv, o);
        if (lane >= o) {
          if (!cr) {
            cv += ycv;
            cr = ycr;
          }
          if (!pr) {
            pv = ypv;
            pr = ypr;
          }
        }
      }
      uint32_t ecr = (uint32_t)__shfl_up((int)cr, 1), ecv = (uint32_t)__shfl_up((int)cv, 1);
      uint32_t epr = (uint32_t)__shfl_up((int)pr, 1), epv = (uint32_t)__shfl_up((int)pv, 1);
      if (lane == 0) ecr = ecv = epr = epv = 0;
      if (live) {
        Seg &sg = segs[s];
        sg.carry_in = ecr ? ecv : carry + ecv;
        sg.prev_dist = epr ? epv : pd;
        sg.extra_ins = 0;
      }
      const uint32_t lcr = (uint32_t)__shfl((int)cr, 63), lcv = (uint32_t)__shfl((int)cv, 63);
      const uint32_t lpr = (uint32_t)__shfl((int)pr, 63), lpv = (uint32_t)__shfl((int)pv, 63);
      carry = lcr ? lcv : carry + lcv;
      pd = lpr ? lpv : pd;
    }
    if (carry && lane == 0) segs[end - 1].extra_ins = carry;
  }
}

// ---------------------------------------------------------------- context mode per metablock
// Native brotli's rule (ChooseContextMode / BrotliIsMostlyUTF8, encode.c; the reference's
// chooseContextMode, context.ts:180-227, samples ASCII / UTF-8 / small-delta patterns instead):
// at q >= 10 UTF8 contexts when at least 3/4 of the metablock's first kCtxScan bytes parse as
// UTF-8, else SIGNED; below q10 UTF8.  The reference's picks cost C4 1.4 % (it took SIGNED for
// enwik-style text: 0.36997 vs 0.36469 with UTF8) and fonts 0.5 % (LSB6 vs SIGNED).
// Values: 0 LSB6, 1 MSB6, 2 UTF8, 3 SIGNED (RFC 7932 section 7.1).  Block (one wave) per
// metablock: the first kCtxScan bytes are staged in LDS and lane t parses bytes [64 t, 64 t + 64)
// from each of the four offsets a parse can enter them at (a sequence is at most 4 bytes);
// lane 0 then chains the 64 pieces from offset 0 -- the serial parse's count exactly (one lane
// parsing 4 KiB of global bytes took 0.4 ms per metablock, r05m).
constexpr int kCtxScan = 4096;
__device__ __forceinline__ int utf8_step(const uint8_t *d, int i, int len, int *ok) {   // BrotliParseAsUTF8
  const int b0 = d[i];
  int n = 1;
  *ok = 0;
  if (b0 < 0x80) {
    *ok = 1;
  } else if ((b0 & 0xE0) == 0xC0 && i + 1 < len && (d[i + 1] & 0xC0) == 0x80) {
    n = 2;
    *ok = (((b0 & 0x1F) << 6) | (d[i + 1] & 0x3F)) >= 0x80;
  } else if ((b0 & 0xF0) == 0xE0 && i + 2 < len && (d[i + 1] & 0xC0) == 0x80 && (d[i + 2] & 0xC0) == 0x80) {
    n = 3;
    *ok = (((b0 & 0x0F) << 12) | ((d[i + 1] & 0x3F) << 6) | (d[i + 2] & 0x3F)) >= 0x800;
  } else if ((b0 & 0xF8) == 0xF0 && i + 3 < len && (d[i + 1] & 0xC0) == 0x80 && (d[i + 2] & 0xC0) == 0x80 &&
             (d[i + 3] & 0xC0) == 0x80) {
    n = 4;
    const int v = ((b0 & 0x07) << 18) | ((d[i + 1] & 0x3F) << 12) | ((d[i + 2] & 0x3F) << 6) | (d[i + 3] & 0x3F);
    *ok = v >= 0x10000 && v <= 0x10FFFF;
  }
  return *ok ? n : 1;
}
__global__ __launch_bounds__(64) void context_mode_kernel(const Job *jobs, Mb *mbs, int nmbs, int force) {
  __shared__ uint8_t d[kCtxScan];
  __shared__ uint16_t cnt[64][4];
  __shared__ uint8_t nxt[64][4];
  const int m = blockIdx.x, t = threadIdx.x;
  if (m >= nmbs) return;
  Mb &mb = mbs[m];
  const Job &jb = jobs[mb.job];
  if (jb.uncompressed) return;
  const uint8_t *src = jb.data + mb.start;
  const int len = (int)min(mb.end - mb.start, (uint32_t)kCtxScan);
  for (int i = t; i < len; i += 64) d[i] = src[i];
  __syncthreads();
  const int c0 = 64 * t, c1 = min(c0 + 64, len);
  for (int e = 0; e < 4; e++) {
    int i = c0 + e, valid = 0, ok;
    while (i < c1) {
      const int n = utf8_step(d, i, len, &ok);
      valid += ok ? n : 0;
      i += n;
    }
    cnt[t][e] = (uint16_t)valid;
    nxt[t][e] = (uint8_t)(i - c1);   // (0..3: where the parse enters the next piece)
  }
  __syncthreads();
  if (t) return;
  int valid = 0, e = 0;
  for (int q = 0; 64 * q < len; q++) {
    valid += cnt[q][e];
    e = nxt[q][e];
  }
  const int mode = !jb.hq || 4 * valid > 3 * len ? 2 : 3;
  mb.ctx_mode = (uint32_t)(force >= 0 ? force : mode);
  if (mb.ctx_mode != 2u) atomicOr(const_cast<uint32_t *>(&jb.binary), 1u);
}

// ---------------------------------------------------------------- codes + unit histograms
// Block per segment: command prefix codes (getInsertLengthCode / getCopyLengthCode /
// combineLengthCodes / prefixEncodeCopyDistance, command.ts:29-179), command positions
// (block scan), and per block-split unit (8 KiB of the segment's commands) its order-0
// literal, command and distance-code histograms, symbol counts and first commands -- the
// symbol streams splitBlock works on (block-splitter.ts:394-464).
template <int NT>
__global__ __launch_bounds__(NT) void codes_kernel(const Job *jobs, const Seg *segs, const Mb *mbs, const RawCmd *raw,
                                                       Cmd *cmds, uint32_t *cmd_pos, Unit *units, uint32_t *unit_h) {
  typedef hipcub::BlockScan<uint64_t, NT> Scan;
  __shared__ typename Scan::TempStorage scan_tmp;
  __shared__ uint32_t sh_h[kSubPerSeg * kSubHist];
  __shared__ uint32_t sh_n[kSubPerSeg][3], sh_first[kSubPerSeg][3];
  __shared__ uint32_t sh_run;
  __shared__ ItemMap<NT> map;
  __shared__ uint32_t sh_pos[NT];
  __shared__ uint32_t sh_push[NT];   // the batch's pushed distances, by rank
  __shared__ uint32_t sh_ring[4];        // the ring before the batch, most recent first
  const Seg sg = segs[blockIdx.x];
  const Job &jb = jobs[sg.job];
  if (jb.uncompressed) return;
  const int t = threadIdx.x;
  for (int i = t; i < kSubPerSeg * kSubHist; i += NT) sh_h[i] = 0;
  if (t < kSubPerSeg * 3) {
    sh_n[t / 3][t % 3] = 0;
    sh_first[t / 3][t % 3] = ~0u;
  }
  if (t == 0) sh_run = sg.start - sg.carry_in;
  // (from global: a lane-indexed read of the by-value copy kept that copy in scratch memory,
  // and every later field read with it)
  if (t < 4) sh_ring[t] = segs[blockIdx.x].ring_in[t];
  __syncthreads();
  const RawCmd *r = raw + sg.cmd_off;
  Cmd *out = cmds + sg.cmd_off;
  uint32_t *outp = cmd_pos + sg.cmd_off;
  const uint32_t nraw = sg.ncmd, n = nraw + (sg.extra_ins ? 1 : 0);
  for (uint32_t base = 0; base < n; base += NT) {
    const uint32_t q = base + t;
    uint32_t ins = 0, len = 0, d = 0, prevd = 0;
    if (q < nraw) {
      const RawCmd rc = r[q];
      ins = rc.ins + (q == 0 ? sg.carry_in : 0);
      len = rc.len;
      d = rc.dist;
      prevd = q ? r[q - 1].dist : sg.prev_dist;
    } else if (q < n) {
      ins = sg.extra_ins;
    }
    // the decoder's distance ring before this command: pushes of the batch before it (by
    // rank), then the ring the batch started with
    const uint32_t push = (q < nraw && !is_word(jb, d) && d != prevd) ? 1u : 0u;   // dictionary words never push
    // one block scan of three packed counts, each field wide enough for its batch total (no
    // carries between fields): bytes, insert + copy, bits 35-63 (< 2^24 carried literals of
    // a <= 16 MiB metablock + the segment); literals, bits 10-34 (< 2^25); ring pushes, bits
    // 0-9 (<= NT)
    static_assert(NT < 1024, "the pushes' field");
    uint64_t ex, tot;
    Scan(scan_tmp).ExclusiveSum(((uint64_t)(ins + len) << 35) | ((uint64_t)ins << 10) | push, ex, tot);
    const uint32_t off = (uint32_t)(ex >> 35), total = (uint32_t)(tot >> 35);
    const uint32_t loff = (uint32_t)(ex >> 10) & 0x1FFFFFFu, nlits = (uint32_t)(tot >> 10) & 0x1FFFFFFu;
    const uint32_t rank = (uint32_t)ex & 0x3FFu, npush = (uint32_t)tot & 0x3FFu;
    const uint32_t pos = sh_run + off;
    if (push) sh_push[rank] = d;
    __syncthreads();
    uint32_t ring[4];
#pragma unroll
    for (int k = 0; k < 4; k++) ring[k] = (int)rank - 1 - k >= 0 ? sh_push[rank - 1 - k] : sh_ring[k - rank];
    uint32_t ring_after = 0;   // the ring after the batch
    if (t < 4) ring_after = (int)npush - 1 - t >= 0 ? sh_push[npush - 1 - t] : sh_ring[t - npush];
    __syncthreads();
    if (t < 4) sh_ring[t] = ring_after;
    if (t == 0) sh_run += total;
    if (q < n) {
      Cmd c;
      c.ins = ins;
      c.copy = len;
      c.dist = d;
      c.dist_extra = 0;
      c.dist_prefix = 0;
      const int ic = ins_code(ins);
      const uint32_t u = unit_of(sg, pos);
      uint32_t *hu = sh_h + u * kSubHist;
      if (len) {
        const uint32_t dcode = is_word(jb, d) ? (d & ~kDictFlag) + 15 : d == prevd ? 0 : short_code(d, ring);
        uint32_t extra;
        const uint32_t dp = dist_prefix(dcode, (int)jb.ndirect, (int)jb.npostfix, &extra);
        c.dist_extra = extra;
        c.dist_prefix = (uint16_t)dp;
        c.cmd_prefix = (uint16_t)combine_codes(ic, copy_code(len), dcode == 0);
        if (c.cmd_prefix >= 128) {
          atomicAdd(&hu[256 + 704 + (dp & 0x3FF)], 1u);
          atomicAdd(&sh_n[u][2], 1u);
          atomicMin(&sh_first[u][2], q);
        }
      } else {   // insert-only: copy code 0 with the implicit last distance when possible
        c.cmd_prefix = (uint16_t)combine_codes(ic, 0, ic < 8);
      }
      atomicAdd(&hu[256 + c.cmd_prefix], 1u);
      atomicAdd(&sh_n[u][1], 1u);
      atomicMin(&sh_first[u][1], q);
      if (ins) {   // literals count to the unit of their own position
        const uint32_t ulo = unit_of(sg, pos), uhi = unit_of(sg, pos + ins - 1);
        for (uint32_t v = ulo; v <= uhi; v++) {
          const uint32_t s0 = v == ulo ? pos : sg.start + (v << kSubBits);
          const uint32_t s1 = v == uhi ? pos + ins : sg.start + ((v + 1) << kSubBits);
          atomicAdd(&sh_n[v][0], s1 - s0);
          atomicMin(&sh_first[v][0], s0);
        }
      }
      out[q] = c;
      outp[q] = pos;
    }
    // the literals of the batch, spread over the lanes (items = inserts, see ItemMap)
    sh_pos[t] = pos;
    const uint32_t nb = min((uint32_t)NT, n - base);
    map.off[t] = loff;
    if (t == 0) map.off[nb] = nlits;
    __syncthreads();
    for (uint32_t i = t; i < nlits; i += NT) {
      const uint32_t j = map.find(i, nb);
      const uint32_t lp = sh_pos[j] + i - map.off[j];
      atomicAdd(&sh_h[unit_of(sg, lp) * kSubHist + jb.data[lp]], 1u);
    }
    __syncthreads();
  }
  const uint32_t u0 = blockIdx.x * kSubPerSeg;
  uint32_t *gh = unit_h + (size_t)u0 * kSubHist;
  for (int i = t; i < kSubPerSeg * kSubHist; i += NT) gh[i] = sh_h[i];
  if (t < kSubPerSeg) {
    Unit un;
    for (int c = 0; c < 3; c++) {
      un.nsym[c] = sh_n[t][c];
      un.first[c] = sh_first[t][c];
      un.sw_count[c] = 0;
      un.type[c] = 0;
      un.sw_code[c] = 0;
    }
    un.pad = 0;
    units[u0 + t] = un;
  }
}

// ---------------------------------------------------------------- histograms by block type
// Block per segment, after the split: literal histograms per (block type, context), command
// histograms per block type, distance-code histograms per (block type, distance context),
// accumulated in LDS (literals one block type at a time) and added to the metablock's with
// one global atomic per non-zero bin (the histogram pass of storeMetaBlock, metablock.ts:580-640).
template <int NT>
__global__ __launch_bounds__(NT) void histo_kernel(const Job *jobs, const Seg *segs, const Mb *mbs, const Cmd *cmds,
                                                       const uint32_t *cmd_pos, const Unit *units, uint32_t *hl,
                                                       uint32_t *hc, uint32_t *hd) {
  typedef hipcub::BlockScan<uint32_t, NT> Scan;
  __shared__ typename Scan::TempStorage scan_tmp;
  __shared__ uint32_t sh_l[kLitCtx * 256];   // command + distance histograms first, then literals per type
  __shared__ uint8_t ut[kSubPerSeg][3];
  __shared__ ItemMap<NT> map;
  __shared__ uint32_t sh_pos[NT], sh_ins[NT];
  uint32_t *sh_c = sh_l, *sh_d = sh_l + kMaxBT * 704;
  const Seg &sg = segs[blockIdx.x];
  const Job &jb = jobs[sg.job];
  if (jb.uncompressed) return;
  const Mb &mb = mbs[sg.mb];
  const int t = threadIdx.x;
  __shared__ uint8_t lut[512];   // the context-mode table, per-literal lookups from LDS
  for (int i = t; i < 512; i += NT) lut[i] = kRfcContextLut[(mb.ctx_mode << 9) + i];
  const Unit *un = units + (size_t)blockIdx.x * kSubPerSeg;
  if (t < kSubPerSeg * 3) ut[t / 3][t % 3] = un[t / 3].type[t % 3];
  for (int i = t; i < (int)mb.nbt[1] * 704; i += NT) sh_c[i] = 0;
  for (int i = t; i < (int)mb.nbt[2] * kDistCtx * 128; i += NT) sh_d[i] = 0;
  __syncthreads();
  const Cmd *c = cmds + sg.cmd_off;
  const uint32_t *cp = cmd_pos + sg.cmd_off;
  const uint32_t n = sg.ncmd + (sg.extra_ins ? 1 : 0);
  for (uint32_t q = t; q < n; q += NT) {
    const Cmd k = c[q];
    const uint32_t u = unit_of(sg, cp[q]);
    atomicAdd(&sh_c[ut[u][1] * 704 + k.cmd_prefix], 1u);
    if (k.copy && k.cmd_prefix >= 128) atomicAdd(&sh_d[(ut[u][2] * kDistCtx + dist_ctx(k.copy)) * 128 + (k.dist_prefix & 0x3FF)], 1u);
  }
  const uint32_t m = sg.mb;
  __syncthreads();
  for (int i = t; i < (int)mb.nbt[1] * 704; i += NT)
    if (sh_c[i]) atomicAdd(&hc[(size_t)m * kMaxBT * 704 + i], sh_c[i]);
  for (int i = t; i < (int)mb.nbt[2] * kDistCtx * 128; i += NT)
    if (sh_d[i]) atomicAdd(&hd[(size_t)m * kMaxBT * kDistCtx * 128 + i], sh_d[i]);
  __syncthreads();
  uint32_t present = 0;   // literal block types used by this segment
  for (int u = 0; u < kSubPerSeg; u++) present |= 1u << ut[u][0];
  for (int ty = 0; ty < kMaxBT; ty++) {
    if (!(present >> ty & 1)) continue;
    for (int i = t; i < kLitCtx * 256; i += NT) sh_l[i] = 0;
    __syncthreads();
    for (uint32_t base = 0; base < n; base += NT) {   // the literals of this type, spread over the lanes
      const uint32_t q = base + t, nb = min((uint32_t)NT, n - base);
      uint32_t cnt = 0;
      if (q < n && c[q].ins) {   // the command's literals that lie in units of this type
        const uint32_t pos = cp[q], ins = c[q].ins;
        sh_pos[t] = pos;
        sh_ins[t] = ins;
        const uint32_t ulo = unit_of(sg, pos), uhi = unit_of(sg, pos + ins - 1);
        for (uint32_t v = ulo; v <= uhi; v++)
          if (ut[v][0] == ty) {
            const uint32_t s0 = v == ulo ? pos : sg.start + (v << kSubBits);
            const uint32_t s1 = v == uhi ? pos + ins : sg.start + ((v + 1) << kSubBits);
            cnt += s1 - s0;
          }
      }
      uint32_t off, nlits;
      Scan(scan_tmp).ExclusiveSum(cnt, off, nlits);
      map.off[t] = off;
      if (t == 0) map.off[nb] = nlits;
      __syncthreads();
      for (uint32_t i = t; i < nlits; i += NT) {
        const uint32_t j = map.find(i, nb);
        // the (i - off)-th of command j's literals in type-ty units (an insert spans few units)
        const uint32_t pos = sh_pos[j], ins = sh_ins[j];
        const uint32_t ulo = unit_of(sg, pos), uhi = unit_of(sg, pos + ins - 1);
        uint32_t k = i - map.off[j], lp = pos;
        for (uint32_t v = ulo; v <= uhi; v++) {
          if (ut[v][0] != ty) continue;
          const uint32_t s0 = v == ulo ? pos : sg.start + (v << kSubBits);
          const uint32_t s1 = v == uhi ? pos + ins : sg.start + ((v + 1) << kSubBits);
          if (k < s1 - s0) {
            lp = s0 + k;
            break;
          }
          k -= s1 - s0;
        }
        const uint32_t p12 = prev2(jb, lp);
        atomicAdd(&sh_l[(lut[p12 & 0xFF] | lut[256 + (p12 >> 8)]) * 256 + jb.data[lp]], 1u);
      }
      __syncthreads();
    }
    uint32_t *dst = hl + ((size_t)m * kLitSlots + ty * kLitCtx) * 256;
    for (int i = t; i < kLitCtx * 256; i += NT)
      if (sh_l[i]) atomicAdd(&dst[i], sh_l[i]);
    __syncthreads();
  }
}

// ---------------------------------------------------------------- clustering
// clusterHistograms (cluster.ts:317-377) restated for one block: the metablock's context
// histograms (64 literal ones over 256 symbols, or 4 distance ones) are merged greedily --
// always the pair whose merge saves the most estimated bits (populationCost-style: Shannon
// bits + a prefix-code header estimate, bit-cost.ts:44-135) -- until no merge saves bits.
// Writes the context map (clusters numbered by first use, as the decoder's IMTF expects
// nothing of it) and the clustered histograms in place.
__device__ __forceinline__ float hist_cost(float bits, int nnz) {
  if (nnz <= 1) return 12.f;
  if (nnz <= 4) return bits + 20.f + 4.f * nnz;
  return bits + 40.f + 3.5f * nnz;
}

// Block per (metablock, literal | distance, block type): the type's context histograms.  A
// literal block type may keep at most lit_cap / (literal block types) codes (launch_cluster):
// past that cap the cheapest merge is taken even when it costs bits.
// 16 waves, and a working set (64 histograms + the a < b pair savings) small enough for two
// blocks per CU (44 VGPRs: 8 waves per SIMD): one block's barriers and LDS round trips in the
// merge loop overlap the other's
constexpr int kCluT = 1024;
constexpr int kCluPairs = kLitCtx * (kLitCtx - 1) / 2;
// pair (a, b), a < b, in the triangular savings table; lexicographic, as a * 64 + b orders them
__device__ __forceinline__ int tri(int a, int b) { return a * (2 * kLitCtx - a - 1) / 2 + b - a - 1; }
#ifdef MIB_PROF   // timing experiment: thread 0's cycles in costs / initial pairs / best-pair search / merges / output; merges
__device__ unsigned long long g_clu_prof[8];
#endif
__global__ __launch_bounds__(kCluT) void cluster_kernel(const Job *jobs, Mb *mbs, int nmbs, uint32_t *hl, uint32_t *hd,
                                                         int lit_cap, int kl, int kd) {
  constexpr int kMaxH = kLitCtx;
  // rows padded by one word: lanes reading one symbol of 64 different histograms hit 64 banks
  __shared__ uint32_t h[kMaxH][257];
  __shared__ float cost[kMaxH];
  __shared__ float save[kCluPairs];
  __shared__ uint16_t pair_of[kCluPairs];   // tri index -> a << 8 | b
  __shared__ int alive[kMaxH], label[kMaxH];
  __shared__ float red_v[kCluT / 64];
  __shared__ int red_i[kCluT / 64];
  __shared__ int sh_best, sh_alive;
  __shared__ int rep_id[kMaxH];
  // block per (metablock, literal type < kl | distance type < 4); distance types 4 .. kd - 1 (the
  // split's widening pass, rarely present) as a second item of the first blocks, so that the
  // launch has no block per absent type (4 more per metablock: +2.7 ms a C4 launch, r06o)
  const int nb = kl + 4, m = blockIdx.x / nb, r0 = blockIdx.x % nb;
  Mb &mb = mbs[m];
  const Job &jb = jobs[mb.job];
  if (jb.uncompressed) return;
  const int t = threadIdx.x;
#ifdef MIB_PROF
  uint64_t cp[6] = {0, 0, 0, 0, 0, 0}, cp0 = __builtin_amdgcn_s_memtime();
#define CLMARK(k)                                         \
  do {                                                    \
    if (t == 0) {                                         \
      const uint64_t t_ = __builtin_amdgcn_s_memtime();   \
      cp[k] += t_ - cp0;                                  \
      cp0 = t_;                                           \
    }                                                     \
  } while (0)
#else
#define CLMARK(k) do {} while (0)
#endif
  auto item = [&](const int kind, const int ty) {
  const int nbt = (int)(kind == 0 ? mb.nbt[0] : mb.nbt[2]);
  if (ty >= nbt) {
    if (t == 0) {
      if (kind == 0) mb.nlit_t[ty] = 0;
      else mb.ndist_t[ty] = 0;
    }
    return;
  }
  const int nh = kind == 0 ? kLitCtx : kDistCtx;
  // The decoder keeps a metablock's prefix codes in its LDS table area (decode.hip kLdsTab,
  // 12,224 entries, at least 257 a code) only when they all fit.  The literal cap is sized for
  // four command and four distance types; each type past four takes room from the literal codes:
  // a command code (704 symbols, ~400 entries with its second-level tables) two literal codes'
  // worth, a distance type (up to four codes) four.  (Past the area a stream still decodes, with
  // every symbol lookup an HBM load: C4 decode 140 -> 299 ms with eight command and distance
  // types and no such budget, r04af.)
  const int extra = 2 * max(0, (int)mb.nbt[1] - 4) + 4 * max(0, (int)mb.nbt[2] - 4);
  const int mb_lit_cap = max((int)mb.nbt[0], lit_cap - extra);
  const int cap = kind == 0 ? max(1, mb_lit_cap / nbt) : kDistCtx;
  const int A = kind == 0 ? 256 : 16 + (int)jb.ndirect + (48 << jb.npostfix);
  const int stride = kind == 0 ? 256 : 128;
  uint32_t *src = kind == 0 ? hl + ((size_t)m * kLitSlots + ty * kLitCtx) * 256
                            : hd + ((size_t)m * kMaxBT * kDistCtx + ty * kDistCtx) * 128;
  for (int i = t; i < nh * 256; i += kCluT) {
    const int a = i / 256, x = i % 256;
    h[a][x] = x < A ? src[a * stride + x] : 0u;
  }
  __syncthreads();
  // each histogram's cost, and which contexts are used at all
  for (int a = t; a < nh; a += kCluT) {
    float sum = 0.f, ent = 0.f;
    int nnz = 0;
    for (int x = 0; x < A; x++) {
      const float c = (float)h[a][x];
      if (c > 0.f) {
        sum += c;
        ent -= c * __log2f(c);
        nnz++;
      }
    }
    if (sum > 0.f) ent += sum * __log2f(sum);
    cost[a] = hist_cost(ent, nnz);
    alive[a] = sum > 0.f ? 1 : 0;
    label[a] = a;
  }
  __syncthreads();
  if (t == 0) {
    int na = 0;
    for (int a = 0; a < nh; a++) na += alive[a];
    sh_alive = na;
  }
  CLMARK(0);
  if (cap == 1 && sh_alive > 1) {
    // one code for the type (the decoder budget left no more, cluster_kernel's caller): every
    // used context merged into the first, no pair search
    __shared__ int sh_a0;
    if (t == 0) {
      int a0 = 0;
      while (!alive[a0]) a0++;
      sh_a0 = a0;
    }
    __syncthreads();
    const int a0 = sh_a0;
    for (int x = t; x < A; x += kCluT) {
      uint32_t v = 0;
      for (int a = 0; a < nh; a++) v += alive[a] ? h[a][x] : 0u;
      h[a0][x] = v;
    }
    __syncthreads();
    if (t < nh && alive[t]) label[t] = a0;
    if (t < nh && t != a0) alive[t] = 0;
    if (t == 0) sh_alive = 1;
    __syncthreads();
  }
  // savings of every pair
  auto pair_saving = [&](int a, int b) -> float {
    float sum = 0.f, ent = 0.f;
    int nnz = 0;
    for (int x = 0; x < A; x++) {
      const float c = (float)(h[a][x] + h[b][x]);
      if (c > 0.f) {
        sum += c;
        ent -= c * __log2f(c);
        nnz++;
      }
    }
    if (sum > 0.f) ent += sum * __log2f(sum);
    return cost[a] + cost[b] - hist_cost(ent, nnz);
  };
  for (int p = t; p < kMaxH * kMaxH; p += kCluT) {
    const int a = p / kMaxH, b = p % kMaxH;
    if (a < b) {
      save[tri(a, b)] = -1e30f;
      pair_of[tri(a, b)] = (uint16_t)(a << 8 | b);
    }
  }
  __syncthreads();
  // only the nh (nh - 1) / 2 pairs a < b, folded into nh / 2 rows of nh - 1: row r holds
  // (r, r+1 .. nh-1) and (nh-1-r, nh-r .. nh-1)
  for (int p = t; p < (nh / 2) * (nh - 1); p += kCluT) {
    const int r = p / (nh - 1), c = p % (nh - 1);
    const int a = c >= r ? r : nh - 1 - r, b = c >= r ? c + 1 : nh - r + c;
    if (alive[a] && alive[b]) save[tri(a, b)] = pair_saving(a, b);
  }
  __syncthreads();
  CLMARK(1);
  for (;;) {
    // best pair
    float bv = -1e30f;
    int bi = -1;
    // the whole table: its index orders pairs as a * nh + b does
    for (int p = t; p < kCluPairs; p += kCluT) {
      const float v = save[p];
      if (v > bv) {
        bv = v;
        bi = p;
      }
    }
    // the largest saving, ties to the lowest pair index: within the wave by shuffles, then
    // one wave over the 16 wave winners
    auto better = [](float v, int i, float bv, int bi) {
      return v > bv || (v == bv && i >= 0 && (bi < 0 || i < bi));
    };
    for (int o = 32; o; o >>= 1) {
      const float v = __shfl_xor(bv, o);
      const int i = __shfl_xor(bi, o);
      if (better(v, i, bv, bi)) {
        bv = v;
        bi = i;
      }
    }
    if ((t & 63) == 0) {
      red_v[t >> 6] = bv;
      red_i[t >> 6] = bi;
    }
    __syncthreads();
    if (t < 64) {
      bv = t < kCluT / 64 ? red_v[t] : -1e30f;
      bi = t < kCluT / 64 ? red_i[t] : -1;
      for (int o = 32; o; o >>= 1) {
        const float v = __shfl_xor(bv, o);
        const int i = __shfl_xor(bi, o);
        if (better(v, i, bv, bi)) {
          bv = v;
          bi = i;
        }
      }
      if (t == 0) sh_best = (bv > 0.f || (sh_alive > cap && bv > -1e29f)) ? bi : -1;
    }
    __syncthreads();
    const int best = sh_best;
    CLMARK(2);
    if (best < 0) break;
#ifdef MIB_PROF
    cp[5]++;
#endif
    const int a = pair_of[best] >> 8, b = pair_of[best] & 0xFF;   // merge b into a
    for (int x = t; x < A; x += kCluT) h[a][x] += h[b][x];
    __syncthreads();
    if (t == 0) {
      cost[a] = cost[a] + cost[b] - save[best];
      alive[b] = 0;
      sh_alive--;
    }
    for (int q = t; q < nh; q += kCluT)
      if (label[q] == b) label[q] = a;
    __syncthreads();
    // pairs with b die; pairs with a change: a wave per pair, lanes over the symbols
    for (int q = t; q < nh; q += kCluT)
      if (q != b) save[tri(min(q, b), max(q, b))] = -1e30f;
    __syncthreads();
    for (int q = t >> 6; q < nh; q += kCluT / 64) {
      if (q == a || q == b) continue;
      const int lo = min(q, a), hi = max(q, a);
      if (!alive[q]) {
        if ((t & 63) == 0) save[tri(lo, hi)] = -1e30f;
        continue;
      }
      float sum = 0.f, ent = 0.f;
      int nnz = 0;
      for (int x = t & 63; x < A; x += 64) {
        const float c = (float)(h[a][x] + h[q][x]);
        if (c > 0.f) {
          sum += c;
          ent -= c * __log2f(c);
          nnz++;
        }
      }
      for (int o = 32; o; o >>= 1) {
        sum += __shfl_xor(sum, o);
        ent += __shfl_xor(ent, o);
        nnz += __shfl_xor(nnz, o);
      }
      if ((t & 63) == 0) {
        if (sum > 0.f) ent += sum * __log2f(sum);
        save[tri(lo, hi)] = cost[lo] + cost[hi] - hist_cost(ent, nnz);
      }
    }
    __syncthreads();
  }
  CLMARK(3);
  // number the clusters by first use; unused contexts go to cluster 0
  if (t == 0) {
    for (int a = 0; a < nh; a++) rep_id[a] = -1;
    int k = 0;
    for (int q = 0; q < nh; q++)
      if (alive[label[q]] && rep_id[label[q]] < 0) rep_id[label[q]] = k++;
    for (int q = 0; q < nh; q++) {
      const int c = alive[label[q]] ? rep_id[label[q]] : 0;
      if (kind == 0) mb.lit_cmap[ty * kLitCtx + q] = (uint16_t)(ty * kLitCtx + c);
      else mb.dist_cmap[ty * kDistCtx + q] = (uint8_t)(ty * kDistCtx + c);
    }
    if (k == 0) k = 1;
    if (kind == 0) mb.nlit_t[ty] = (uint32_t)k;
    else mb.ndist_t[ty] = (uint32_t)k;
  }
  __syncthreads();
  // clustered histograms, in place: cluster c <- its representative's merged histogram
  for (int i = t; i < nh * stride; i += kCluT) src[i] = 0;
  __syncthreads();
  for (int i = t; i < nh * 256; i += kCluT) {
    const int a = i / 256, x = i % 256;
    const int c = alive[a] ? rep_id[a] : -1;
    if (c >= 0 && x < A) src[c * stride + x] = h[a][x];
  }
  };
  item(r0 < kl ? 0 : 1, r0 < kl ? r0 : r0 - kl);
  if (r0 < kd - 4) {
    __syncthreads();
    item(1, 4 + r0);
  }
#ifdef MIB_PROF
  CLMARK(4);
  if (t == 0)
    for (int q = 0; q < 6; q++) atomicAdd(&g_clu_prof[q], (unsigned long long)cp[q]);
  if (t == 0) atomicAdd(&g_clu_prof[6], 1ull);
#endif
#undef CLMARK
}

// ---------------------------------------------------------------- distance ring after a chunk
// (streaming: the next chunk's code-0 decisions start from it) lane per stream, backwards
// over the last commands: every explicit distance was pushed.
__global__ void dist_ring_kernel(Job *jobs, int njobs, const Seg *segs, const Cmd *cmds) {
  int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= njobs) return;
  Job &jb = jobs[j];
  if (jb.uncompressed) return;
  int32_t ring[4];
  int got = 0;
  for (int s = (int)(jb.seg_base + jb.nseg) - 1; s >= (int)jb.seg_base && got < 4; s--) {
    const Seg &sg = segs[s];
    const Cmd *c = cmds + sg.cmd_off;
    for (int q = (int)sg.ncmd - 1; q >= 0 && got < 4; q--)
      if ((c[q].dist_prefix & 0x3FF) != 0 && !is_word(jb, c[q].dist)) ring[got++] = (int32_t)c[q].dist;
  }
  for (int q = 0; q < 4; q++) jb.dc_out[q] = q < got ? ring[q] : jb.dc_in[q - got];
}

// ---------------------------------------------------------------- Huffman codes
// Block (one wave) per (metablock, alphabet).  createHuffmanTree (entropy-encode.ts:24-131):
// leaves sorted by (count ascending, symbol descending) -- ranks computed by the 64 lanes --
// two-queue merge and depth walk by lane 0, count-limit doubling until depth <= 15;
// convertBitDepthsToSymbols (:234-258); buildAndStoreHuffmanTree simple / complex forms
// (context-map.ts:215-347).
__device__ void tree_depths(const uint32_t *h, const int16_t *sorted, int n, uint32_t lc, int limit, uint8_t *depth,
                            uint32_t *cnt, int16_t *left, int16_t *val, bool *ok) {
  for (int k = 0; k < n; k++) {
    uint32_t c = h[sorted[k]];
    cnt[k] = c > lc ? c : lc;
    left[k] = -1;
    val[k] = sorted[k];
  }
  cnt[n] = cnt[n + 1] = 0xFFFFFFFFu;
  left[n] = left[n + 1] = -1;
  val[n] = val[n + 1] = -1;
  int i = 0, j = n + 1;
  for (int k = n - 1; k > 0; k--) {
    int l, r;
    if (cnt[i] <= cnt[j]) l = i++; else l = j++;
    if (cnt[i] <= cnt[j]) r = i++; else r = j++;
    const int je = 2 * n - k;
    cnt[je] = cnt[l] + cnt[r];
    left[je] = (int16_t)l;
    val[je] = (int16_t)r;
    cnt[je + 1] = 0xFFFFFFFFu;
    left[je + 1] = -1;
    val[je + 1] = -1;
  }
  int16_t stack[18];
  int level = 0, p = 2 * n - 1;
  stack[0] = -1;
  *ok = true;
  for (;;) {
    if (left[p] >= 0) {
      level++;
      if (level > limit) {
        *ok = false;
        return;
      }
      stack[level] = val[p];
      p = left[p];
      continue;
    }
    depth[val[p]] = (uint8_t)level;
    while (level >= 0 && stack[level] == -1) level--;
    if (level < 0) return;
    p = stack[level];
    stack[level] = -1;
  }
}

// tree_depths for the Huffman kernel's codes, by the wave (all 64 lanes call it; the same depths
// and the same success test): the leaf counts are clamped by the wave; lane 0 runs the two-queue
// merge with the heads of both queues and the entries after them in registers -- each step's
// compares wait for no LDS read, the next entries load behind them -- and records parent links;
// the internal nodes' depths follow by one walk down from the root (a parent's index is above
// its children's), the leaves' by the wave.  (The serial merge and the stack walk re-read every
// node from LDS: 1.2 M cycles for the largest code of a 1 MiB metablock, r05ah.)
// par / dint: 2n entries each.
__device__ bool tree_depths_wave(const uint32_t *h, const int16_t *sorted, int n, uint32_t lc, int limit, uint8_t *depth,
                                 uint32_t *cnt, int16_t *par, int16_t *dint) {
  const int lane = threadIdx.x & 63;
  constexpr uint32_t kInfC = 0xFFFFFFFFu;
  for (int k = lane; k < n; k += 64) {
    const uint32_t c = h[sorted[k]];
    cnt[k] = c > lc ? c : lc;
  }
  wave_sync();
  if (lane == 0) {
    // leaves 0 .. n-1, internal nodes n+1 .. 2n-1 in creation order (tree_depths' layout); a
    // queue's head and the entry after it: leaves a, a2 (at i, i + 1), internal b, b2 (at j,
    // j + 1), an entry not there (yet) being "infinite"; ties take the leaf
    int i = 0, j = n + 1, made = n;
    uint32_t a = cnt[0], a2 = n > 1 ? cnt[1] : kInfC, b = kInfC, b2 = kInfC;
    for (int k = n - 1; k > 0; k--) {
      const int je = 2 * n - k;
      int l, r;
      uint32_t cl, cr;
      if (a <= b) {
        l = i++;
        cl = a;
        a = a2;
        a2 = i + 1 < n ? cnt[i + 1] : kInfC;
      } else {
        l = j++;
        cl = b;
        b = b2;
        b2 = j + 1 <= made ? cnt[j + 1] : kInfC;
      }
      if (a <= b) {
        r = i++;
        cr = a;
        a = a2;
        a2 = i + 1 < n ? cnt[i + 1] : kInfC;
      } else {
        r = j++;
        cr = b;
        b = b2;
        b2 = j + 1 <= made ? cnt[j + 1] : kInfC;
      }
      const uint32_t sum = cl + cr;
      cnt[je] = sum;
      par[l] = (int16_t)je;
      par[r] = (int16_t)je;
      made = je;
      if (j == je) b = sum;
      else if (j + 1 == je) b2 = sum;
    }
    dint[2 * n - 1] = 0;   // the root
    for (int x = 2 * n - 2; x > n; x--) dint[x] = (int16_t)(dint[par[x]] + 1);
  }
  wave_sync();
  int mx = 0;
  for (int k = lane; k < n; k += 64) {
    const int d = dint[par[k]] + 1;
    depth[sorted[k]] = (uint8_t)d;
    mx = max(mx, d);
  }
#pragma unroll
  for (int o = 32; o; o >>= 1) mx = max(mx, __shfl_xor(mx, o));
  wave_sync();
  return mx <= limit;
}

// Scratch of the serial tree helpers.  The Huffman kernel keeps one in LDS: as private arrays
// (dynamically indexed, so in scratch memory) they made serialising a code cost ~600-850 K
// cycles -- most of the kernel (r03m, scripts/huff_timing.py).
struct TreeScratch {
  uint8_t rle_code[720], rle_extra[720];
  uint32_t clh[18];
  uint8_t cld[18];
  uint16_t clc[18];
  int16_t sorted[18];
  int16_t left[40], val[40];
  uint32_t cnt[40];
  uint32_t bl[16], next[16];
};
__device__ void depths_to_codes(const uint8_t *depth, int len, uint16_t *code, uint32_t *bl, uint32_t *next) {
  for (int i = 0; i < 16; i++) bl[i] = next[i] = 0;
  for (int i = 0; i < len; i++) bl[depth[i]]++;
  bl[0] = 0;
  uint32_t c = 0;
  for (int i = 1; i <= 15; i++) {
    c = (c + bl[i - 1]) << 1;
    next[i] = c;
  }
  for (int i = 0; i < len; i++) {
    code[i] = 0;
    if (!depth[i]) continue;
    uint32_t v = next[depth[i]]++, r = 0;
    for (int b = 0; b < depth[i]; b++) r |= ((v >> b) & 1) << (depth[i] - 1 - b);
    code[i] = (uint16_t)r;
  }
}
__device__ void depths_to_codes(const uint8_t *depth, int len, uint16_t *code) {
  uint32_t bl[16], next[16];
  depths_to_codes(depth, len, code, bl, next);
}

// small serial Huffman for the 18 code-length codes (limit 5)
__device__ void small_depths(const uint32_t *h, int len, int limit, uint8_t *depth, TreeScratch &ts) {
  int16_t *sorted = ts.sorted;
  uint32_t *cnt = ts.cnt;
  int16_t *left = ts.left, *val = ts.val;
  for (int i = 0; i < len; i++) depth[i] = 0;
  int n = 0;
  for (int i = len - 1; i >= 0; i--)
    if (h[i]) sorted[n++] = (int16_t)i;
  if (n == 0) return;
  if (n == 1) {
    depth[sorted[0]] = 1;
    return;
  }
  for (uint32_t lc = 1;; lc *= 2) {
    // insertion sort: count ascending, value descending
    for (int a = 1; a < n; a++) {
      int16_t v = sorted[a];
      uint32_t cv = h[v] > lc ? h[v] : lc;
      int k = a - 1;
      while (k >= 0) {
        uint32_t ck = h[sorted[k]] > lc ? h[sorted[k]] : lc;
        if (ck > cv || (ck == cv && sorted[k] < v)) {
          sorted[k + 1] = sorted[k];
          k--;
        } else {
          break;
        }
      }
      sorted[k + 1] = v;
    }
    bool ok;
    tree_depths(h, sorted, n, lc, limit, depth, cnt, left, val, &ok);
    if (ok) return;
    for (int i = 0; i < len; i++) depth[i] = 0;
  }
}

__device__ void put_varlen_u8(BitW &w, int n) {
  if (n == 0) {
    w.put(1, 0);
  } else {
    int nb = 31 - __clz(n);
    w.put(1, 1);
    w.put(3, (uint32_t)nb);
    w.put(nb, (uint32_t)(n - (1 << nb)));
  }
}

// complex prefix code serialisation: run-length code the depths (16 / 17), then a
// depth-5 code for those (writeHuffmanTree / storeHuffmanTreeOfHuffmanTree)
// The run-length codes of depth[0 .. nl) into ts.rle_code / rle_extra; returns their number
__device__ __forceinline__ int rle_depths(const uint8_t *depth, int nl, TreeScratch &ts) {
  uint8_t *rle_code = ts.rle_code, *rle_extra = ts.rle_extra;
  int nr = 0;
  int prev = 8;
  for (int i = 0; i < nl;) {
    int v = depth[i], reps = 1;
    while (i + reps < nl && depth[i + reps] == v) reps++;
    i += reps;
    if (v == 0) {
      if (reps == 11) {
        rle_code[nr] = 0;
        rle_extra[nr++] = 0;
        reps--;
      }
      if (reps < 3) {
        for (int q = 0; q < reps; q++) {
          rle_code[nr] = 0;
          rle_extra[nr++] = 0;
        }
      } else {
        int s0 = nr;
        reps -= 3;
        for (;;) {
          rle_code[nr] = 17;
          rle_extra[nr++] = (uint8_t)(reps & 7);
          reps >>= 3;
          if (!reps) break;
          reps--;
        }
        for (int x = s0, y = nr - 1; x < y; x++, y--) {
          uint8_t tt = rle_code[x]; rle_code[x] = rle_code[y]; rle_code[y] = tt;
          tt = rle_extra[x]; rle_extra[x] = rle_extra[y]; rle_extra[y] = tt;
        }
      }
    } else {
      if (prev != v) {
        rle_code[nr] = (uint8_t)v;
        rle_extra[nr++] = 0;
        reps--;
      }
      if (reps == 7) {
        rle_code[nr] = (uint8_t)v;
        rle_extra[nr++] = 0;
        reps--;
      }
      if (reps < 3) {
        for (int q = 0; q < reps; q++) {
          rle_code[nr] = (uint8_t)v;
          rle_extra[nr++] = 0;
        }
      } else {
        int s0 = nr;
        reps -= 3;
        for (;;) {
          rle_code[nr] = 16;
          rle_extra[nr++] = (uint8_t)(reps & 3);
          reps >>= 2;
          if (!reps) break;
          reps--;
        }
        for (int x = s0, y = nr - 1; x < y; x++, y--) {
          uint8_t tt = rle_code[x]; rle_code[x] = rle_code[y]; rle_code[y] = tt;
          tt = rle_extra[x]; rle_extra[x] = rle_extra[y]; rle_extra[y] = tt;
        }
      }
      prev = v;
    }
  }
  return nr;
}
__device__ const uint8_t kClOrder[18] = {1, 2, 3, 4, 0, 5, 17, 6, 16, 7, 8, 9, 10, 11, 12, 13, 14, 15};
__device__ const uint8_t kClSym[6] = {0, 7, 3, 2, 1, 15}, kClLen[6] = {2, 4, 3, 2, 2, 4};
// The code-length code of the histogram ts.clh (limit 5) and its header part: HSKIP and the
// stored code lengths (storeHuffmanTreeOfHuffmanTree); leaves ts.cld / ts.clc for the symbols
__device__ __forceinline__ void put_cl_code(BitW &w, TreeScratch &ts) {
  uint32_t *clh = ts.clh;
  int ncodes = 0, first = 0;
  for (int k = 0; k < 18; k++)
    if (clh[k]) {
      if (!ncodes) first = k;
      ncodes++;
    }
  uint8_t *cld = ts.cld;
  uint16_t *clc = ts.clc;
  small_depths(clh, 18, 5, cld, ts);
  depths_to_codes(cld, 18, clc, ts.bl, ts.next);
  // (tables in constant memory: as local arrays indexed by data they were copied to scratch)
  const uint8_t *order = kClOrder, *sym = kClSym, *blen = kClLen;
  int to_store = 18;
  if (ncodes > 1)
    while (to_store > 0 && cld[order[to_store - 1]] == 0) to_store--;
  int skip = 0;
  if (cld[order[0]] == 0 && cld[order[1]] == 0) {
    skip = 2;
    if (cld[order[2]] == 0) skip = 3;
  }
  w.put(2, (uint32_t)skip);
  for (int k = skip; k < to_store; k++) {
    int l = cld[order[k]];
    w.put(blen[l], sym[l]);
  }
  if (ncodes == 1) cld[first] = 0;
}
__device__ void store_complex(BitW &w, const uint8_t *depth, int asize, TreeScratch &ts) {
  int nl = asize;
  while (nl > 0 && depth[nl - 1] == 0) nl--;
  const int nr = rle_depths(depth, nl, ts);
  uint32_t *clh = ts.clh;
  for (int k = 0; k < 18; k++) clh[k] = 0;
  for (int k = 0; k < nr; k++) clh[ts.rle_code[k]]++;
  put_cl_code(w, ts);
  for (int k = 0; k < nr; k++) {
    int c = ts.rle_code[k];
    w.put(ts.cld[c], ts.clc[c]);
    if (c == 16) w.put(2, ts.rle_extra[k]);
    else if (c == 17) w.put(3, ts.rle_extra[k]);
  }
}
// Bits of `count` items by the wave at lane 0's writer position (all 64 lanes call it; lane 0
// has flushed w): item k's (bits, value) from item(k), placed by a wave prefix sum and ORed into
// the zeroed, 4-byte-aligned buffer; every lane's w then continues after them.
template <class F>
__device__ void wave_put_items(BitW &w, uint32_t *buf32, int count, F item) {
  const int lane = threadIdx.x & 63;
  uint64_t pos = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)w.pos) |
                 ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(w.pos >> 32)) << 32);
  for (int k0 = 0; k0 < count; k0 += 64) {
    const int k = k0 + lane;
    uint32_t nb = 0, v = 0;
    if (k < count) item(k, nb, v);
    uint32_t incl = nb;   // inclusive prefix sum of the items' bit counts
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = (uint32_t)__shfl_up((int)incl, o);
      if (lane >= o) incl += y;
    }
    if (nb) {
      const uint64_t b = pos + incl - nb;
      const uint32_t wi = (uint32_t)(b >> 5), sh = (uint32_t)(b & 31);
      const uint64_t x = (uint64_t)v << sh;
      atomicOr(buf32 + wi, (uint32_t)x);
      if (sh + nb > 32) atomicOr(buf32 + wi + 1, (uint32_t)(x >> 32));
    }
    pos += (uint32_t)__shfl((int)incl, 63);
  }
  wave_sync();
  w.pos = pos;
  w.acc = 0;
  w.nacc = 0;
}
// store_complex with the wave (all 64 lanes call it; w is lane 0's writer, the others' copies
// follow its position): the last used symbol by ballots, the run-length codes' histogram by LDS
// atomics, and their bits -- each lane one code's, placed by a wave prefix sum and ORed into the
// 4-byte-aligned buffer -- around lane 0's serial run-length coding and code-length code.
// (Serially, the scan, the histogram and the writes were three dependent LDS round trips a
// code: ~2/3 of a 704-symbol code's 0.6 M cycles, r05ai.)
__device__ void store_complex_wave(BitW &w, const uint8_t *depth, int asize, TreeScratch &ts, uint32_t *buf32, int *sh_nr) {
  const int lane = threadIdx.x & 63;
  int nl = 0;
  for (int x0 = (asize - 1) & ~63; x0 >= 0; x0 -= 64) {
    const int x = x0 + lane;
    const uint64_t m = __ballot(x < asize && depth[x] != 0);
    if (m) {
      nl = x0 + 64 - __clzll((long long)m);
      break;
    }
  }
  if (lane < 18) ts.clh[lane] = 0;
  if (lane == 0) *sh_nr = rle_depths(depth, nl, ts);
  wave_sync();
  const int nr = *sh_nr;
  for (int k = lane; k < nr; k += 64) atomicAdd(&ts.clh[ts.rle_code[k]], 1u);
  wave_sync();
  if (lane == 0) {
    put_cl_code(w, ts);
    w.flush();
  }
  wave_sync();
  wave_put_items(w, buf32, nr, [&](int k, uint32_t &nb, uint32_t &v) {
    const int c = ts.rle_code[k];
    const uint32_t d = ts.cld[c], ne = c == 16 ? 2u : c == 17 ? 3u : 0u;
    nb = d + ne;
    v = (uint32_t)ts.clc[c] | ((uint32_t)ts.rle_extra[k] << d);
  });
}

// One prefix code: simple form for up to 4 used symbols (zero-length codeword for one),
// complex form otherwise (buildAndStoreHuffmanTree, context-map.ts:215-347).  `depth`
// holds the code lengths (computed by the caller for n >= 2); `code` is filled.
__device__ void store_code(BitW &w, int n, const int16_t *nzs, int max_bits, uint8_t *depth, uint16_t *code, int asize,
                           TreeScratch &ts, bool codes_done) {
  if (n <= 1) {
    w.put(4, 1);
    w.put(max_bits, n ? (uint32_t)nzs[0] : 0u);
    if (n) depth[nzs[0]] = 0;
    for (int i = 0; i < asize; i++) code[i] = 0;
    return;
  }
  if (!codes_done) depths_to_codes(depth, asize, code, ts.bl, ts.next);
  if (n <= 4) {
    int s4[4];
    for (int i = 0; i < n; i++) s4[i] = nzs[i];
    for (int i = 1; i < n; i++) {
      int v = s4[i], k = i;
      while (k > 0 && depth[s4[k - 1]] > depth[v]) {
        s4[k] = s4[k - 1];
        k--;
      }
      s4[k] = v;
    }
    w.put(2, 1);
    w.put(2, (uint32_t)(n - 1));
    for (int i = 0; i < n; i++) w.put(max_bits, (uint32_t)s4[i]);
    if (n == 4) w.put(1, depth[s4[0]] == 1 ? 1 : 0);
    return;
  }
  store_complex(w, depth, asize, ts);
}
__device__ void store_code(BitW &w, int n, const int16_t *nzs, int max_bits, uint8_t *depth, uint16_t *code, int asize) {
  TreeScratch ts;
  store_code(w, n, nzs, max_bits, depth, code, asize, ts, false);
}

// serial length-limited Huffman depths for small alphabets (<= 80 symbols); the work arrays
// in `ws` (LDS in the header kernel: private arrays indexed by data live in scratch memory)
struct SerialWs {
  int16_t sorted[80];
  uint32_t cnt[2 * 80 + 2];
  int16_t left[2 * 80 + 2], val[2 * 80 + 2];
  int16_t nz[80];   // (serial_depths_wave: the used symbols)
  int n;
};
__device__ void serial_depths(const uint32_t *h, int len, int limit, uint8_t *depth, SerialWs &ws) {
  int16_t *sorted = ws.sorted, *left = ws.left, *val = ws.val;
  uint32_t *cnt = ws.cnt;
  for (int i = 0; i < len; i++) depth[i] = 0;
  int n = 0;
  for (int i = len - 1; i >= 0; i--)
    if (h[i]) sorted[n++] = (int16_t)i;
  if (n == 0) return;
  if (n == 1) {
    depth[sorted[0]] = 1;
    return;
  }
  for (uint32_t lc = 1;; lc *= 2) {
    for (int a = 1; a < n; a++) {   // count ascending, symbol descending
      int16_t v = sorted[a];
      uint32_t cv = h[v] > lc ? h[v] : lc;
      int k = a - 1;
      while (k >= 0) {
        uint32_t ck = h[sorted[k]] > lc ? h[sorted[k]] : lc;
        if (ck > cv || (ck == cv && sorted[k] < v)) {
          sorted[k + 1] = sorted[k];
          k--;
        } else {
          break;
        }
      }
      sorted[k + 1] = v;
    }
    bool ok;
    tree_depths(h, sorted, n, lc, limit, depth, cnt, left, val, &ok);
    if (ok) return;
    for (int i = 0; i < len; i++) depth[i] = 0;
  }
}
__device__ void serial_depths(const uint32_t *h, int len, int limit, uint8_t *depth) {
  SerialWs ws;
  serial_depths(h, len, limit, depth, ws);
}
// serial_depths by the wave (all 64 lanes call it; the same depths): the used symbols compacted
// by ballots, ranked by (clamped count, descending symbol) with every lane comparing its symbols
// against all keys, the tree by tree_depths_wave.  (Serially the insertion sort alone re-read two
// LDS words per step: ~0.4 M cycles for an 80-symbol context-map code, r05.)
__device__ void serial_depths_wave(const uint32_t *h, int len, int limit, uint8_t *depth, SerialWs &ws) {
  const int lane = threadIdx.x & 63;
  int n = 0;
  for (int c0 = 0; c0 < len; c0 += 64) {
    const int i = c0 + lane;
    const bool f = i < len && h[i] != 0;
    const uint64_t m = __ballot(f);
    if (i < len) depth[i] = 0;
    if (f) ws.nz[n + __popcll(m & ((1ull << lane) - 1))] = (int16_t)i;
    n += __popcll(m);
  }
  wave_sync();
  if (n == 0) return;
  if (n == 1) {
    if (lane == 0) depth[ws.nz[0]] = 1;
    wave_sync();
    return;
  }
  uint64_t *keys = reinterpret_cast<uint64_t *>(ws.cnt);   // (80 keys; the tree reuses cnt after the sort)
  static_assert(sizeof(ws.cnt) >= 80 * sizeof(uint64_t), "the sort keys fit cnt");
  for (uint32_t lc = 1;; lc *= 2) {
    uint64_t mine[2] = {~0ull, ~0ull};
    int16_t ms[2] = {0, 0};
#pragma unroll
    for (int q = 0; q < 2; q++) {
      const int a = lane + 64 * q;
      if (a < n) {
        const int si = ws.nz[a];
        const uint32_t ci = h[si] > lc ? h[si] : lc;
        mine[q] = ((uint64_t)ci << 16) | (uint32_t)(0xFFFF - si);
        ms[q] = (int16_t)si;
        keys[a] = mine[q];
      }
    }
    wave_sync();
    uint32_t rk[2] = {0u, 0u};
    for (int b = 0; b < n; b++) {
      const uint64_t kb = keys[b];
      rk[0] += kb < mine[0] ? 1u : 0u;
      rk[1] += kb < mine[1] ? 1u : 0u;
    }
    wave_sync();   // (the keys are read before the tree overwrites cnt)
#pragma unroll
    for (int q = 0; q < 2; q++)
      if (lane + 64 * q < n) ws.sorted[rk[q]] = ms[q];
    wave_sync();
    if (tree_depths_wave(h, ws.sorted, n, lc, limit, depth, ws.cnt, ws.val, ws.left)) return;
    for (int i = lane; i < len; i += 64) depth[i] = 0;
    wave_sync();
  }
}

// Block (one wave) per (metablock, code slot): literal (block type, cluster), command (block
// type), distance (block type, cluster); slots beyond the metablock's counts are empty.
// blocks per metablock: the used codes only (literal codes are at most kMaxLitTrees in all)
#ifdef MIB_PROF   // timing experiment: trees, count-limit attempts, cycles in rank sort / tree / store, per block
__device__ unsigned long long g_huff_prof[12];   // + maxima: block, sort, tree, store cycles
#define HPT() __builtin_amdgcn_s_memtime()
#else
#define HPT() 0ull
#endif
// AMAX: the largest alphabet the launch builds codes for -- 256 for the literal slots, 704 for
// the command and distance ones: the literal codes (most of a metablock's) then need ~10 KiB of
// LDS instead of ~22, so twice as many of these latency-bound one-wave blocks share a CU.
// r0: the first slot block of the launch (block r of metablock m = blockIdx.x / nr, r0 + x % nr)
template <int AMAX>
__global__ __launch_bounds__(64) void huffman_kernel(const Job *jobs, Mb *mbs, int nmbs, const uint32_t *hl,
                                                     const uint32_t *hc, const uint32_t *hd, Codes *codes,
                                                     uint8_t *trees, int nl, int kc, int nr) {
  __shared__ uint32_t h[AMAX];
  __shared__ int16_t nzs[AMAX];
  __shared__ int16_t sorted[AMAX];
  __shared__ __attribute__((aligned(16))) uint32_t cnt[2 * AMAX + 2];   // (also the sort's keys: 8 B each)
  static_assert((2 * AMAX + 2) * 4 >= AMAX * 8, "the sort keys fit cnt");
  __shared__ int16_t left[2 * AMAX + 2], val[2 * AMAX + 2];
  __shared__ uint8_t depth[AMAX];
  __shared__ uint16_t code[AMAX];
  __shared__ __attribute__((aligned(16))) uint8_t buf[kTreeBytes];   // (words for store_complex_wave)
  __shared__ int sh_nr;
  __shared__ TreeScratch ts;
  // nr blocks per metablock: nl literal codes, four command and sixteen distance slots (types
  // 0..3); the slots of command / distance types 4..7 (the split's widening pass, rarely
  // present) are second items of the first blocks, so the launch has no block per absent type
  const int m = blockIdx.x / nr, r = (int)(blockIdx.x % nr);
  const int lane = threadIdx.x;
  Mb &mb = mbs[m];
  const Job &jb = jobs[mb.job];
  if (jb.uncompressed) return;
  auto slot_used = [&](int q) {
    const bool l = q < kCmdSlot, d = q >= kDistSlot;
    const int c = l ? q : d ? q - kDistSlot : q - kCmdSlot;
    return l ? (c / kLitCtx < (int)mb.nbt[0] && c % kLitCtx < (int)mb.nlit_t[c / kLitCtx])
             : d ? (c / kDistCtx < (int)mb.nbt[2] && c % kDistCtx < (int)mb.ndist_t[c / kDistCtx]) : c < (int)mb.nbt[1];
  };
  // the unused slots' sizes are zeroed by the blocks in turn (each slot by one block)
  if (lane == 0)
    for (int q = r; q < kTreeSlots; q += nr)
      if (!slot_used(q)) mb.tree_bits[q] = 0;
  // block r builds the r-th used code: literal codes first (at most kMaxLitTrees of them,
  // numbered per block type), then the command codes, then the distance codes
  int t0 = -1, t1 = -1;
  if (r < nl) {
    int acc = 0;
    for (int ty = 0; ty < (int)mb.nbt[0] && t0 < 0; ty++) {
      if (r < acc + (int)mb.nlit_t[ty]) t0 = ty * kLitCtx + (r - acc);
      acc += (int)mb.nlit_t[ty];
    }
  } else if (r < nl + 4) {
    t0 = kCmdSlot + (r - nl);
  } else {
    t0 = kDistSlot + (r - nl - 4);
  }
  if (r < kc - 4) t1 = kCmdSlot + 4 + r;
  else if (r < kc - 4 + 4 * kDistCtx) t1 = kDistSlot + 4 * kDistCtx + (r - (kc - 4));
  auto item = [&](const int t) {
  if (t < 0 || !slot_used(t)) return;
  const bool lit = t < kCmdSlot, dist = t >= kDistSlot;
  const int cl = lit ? t : dist ? t - kDistSlot : t - kCmdSlot;   // slot within its alphabet
  const int asize = lit ? 256 : !dist ? 704 : 16 + (int)jb.ndirect + (48 << jb.npostfix);
  if (asize > AMAX) return;   // (cannot happen: the literal launch covers the literal slots only)
  const uint32_t *src = lit ? hl + ((size_t)m * kLitSlots + cl) * 256 : !dist ? hc + ((size_t)m * kMaxBT + cl) * 704
                                                                          : hd + ((size_t)m * kMaxBT * kDistCtx + cl) * 128;
  for (int i = lane; i < asize; i += 64) {
    h[i] = src[i];
    depth[i] = 0;
    code[i] = 0;
  }
  for (int i = lane; i < kTreeBytes; i += 64) buf[i] = 0;
  wave_sync();
  // compact the used symbols (ascending)
  int n = 0;
  for (int c0 = 0; c0 < asize; c0 += 64) {
    const int i = c0 + lane;
    const bool f = i < asize && h[i] != 0;
    const uint64_t mask = __ballot(f);
    if (f) nzs[n + __popcll(mask & ((1ull << lane) - 1))] = (int16_t)i;
    n += __popcll(mask);
  }
  wave_sync();
  int max_bits = 0;
  for (int c = asize - 1; c; c >>= 1) max_bits++;
  uint64_t hp0 = HPT(), hp_sort = 0, hp_tree = 0, hp_att = 0;
  if (n > 1) {
    for (uint32_t lc = 1;; lc *= 2) {
      hp_att++;
      const uint64_t ta = HPT();
      // rank sort by (clamped count, descending symbol): key (count << 16) | (0xFFFF - symbol),
      // a symbol's rank = the keys below its own.  The keys in LDS (cnt's space: the tree is
      // built after the sort), read two at a time and compared with all of a lane's symbols
      // (one pair read per two keys, not two reads per key and symbol)
      uint64_t *keys = reinterpret_cast<uint64_t *>(cnt);
      for (int a = lane; a < ((n + 1) & ~1); a += 64) {
        uint64_t k = ~0ull;   // (the pad: below no key)
        if (a < n) {
          const int si = nzs[a];
          const uint32_t ci = h[si] > lc ? h[si] : lc;
          k = ((uint64_t)ci << 16) | (uint32_t)(0xFFFF - si);
        }
        keys[a] = k;
      }
      wave_sync();
      constexpr int kPerLane = (AMAX + 63) / 64;
      uint64_t mine[kPerLane];
      uint32_t rk[kPerLane];
#pragma unroll
      for (int q = 0; q < kPerLane; q++) {
        const int a = lane + 64 * q;
        mine[q] = a < n ? keys[a] : 0ull;
        rk[q] = 0;
      }
      const ulonglong2 *kp = reinterpret_cast<const ulonglong2 *>(keys);
      for (int b = 0; b < n; b += 2) {
        const ulonglong2 kb = kp[b >> 1];
#pragma unroll
        for (int q = 0; q < kPerLane; q++) rk[q] += (uint32_t)(kb.x < mine[q]) + (uint32_t)(kb.y < mine[q]);
      }
#pragma unroll
      for (int q = 0; q < kPerLane; q++) {
        const int a = lane + 64 * q;
        if (a < n) sorted[rk[q]] = nzs[a];
      }
      wave_sync();
      const uint64_t tb = HPT();
      hp_sort += tb - ta;
      const bool ok = tree_depths_wave(h, sorted, n, lc, 15, depth, cnt, val, left);
      if (!ok)
        for (int i = lane; i < asize; i += 64) depth[i] = 0;
      wave_sync();
      hp_tree += HPT() - tb;
      if (ok) break;
    }
  }
  const uint64_t tc = HPT();
  if (n > 1) {
    // canonical codes (convertBitDepthsToSymbols, entropy-encode.ts:234-258) by the wave: the
    // codes of each length in symbol order, 64 symbols a step
    uint32_t cntd = 0;   // lane d (1..15): symbols of length d
    for (int c0 = 0; c0 < asize; c0 += 64) {
      const int i = c0 + lane;
      const int d = i < asize ? depth[i] : 0;
#pragma unroll
      for (int dd = 1; dd <= 15; dd++) {
        const uint64_t m = __ballot(d == dd);   // (every lane: a ballot inside a lane-dependent select would see one lane)
        cntd += lane == dd ? (uint32_t)__popcll(m) : 0u;
      }
    }
    uint32_t nextd = 0, c = 0;   // lane d: the first code of length d
#pragma unroll
    for (int dd = 1; dd <= 15; dd++) {
      c = (c + (uint32_t)__shfl((int)cntd, dd - 1)) << 1;
      nextd = lane == dd ? c : nextd;
    }
    if (lane == 0) nextd = 0;
    for (int c0 = 0; c0 < asize; c0 += 64) {
      const int i = c0 + lane;
      const int d = i < asize ? depth[i] : 0;
      uint32_t v = 0;
#pragma unroll
      for (int dd = 1; dd <= 15; dd++) {
        const uint64_t m = __ballot(d == dd);
        const uint32_t base = (uint32_t)__shfl((int)nextd, dd);
        if (d == dd) v = base + (uint32_t)__popcll(m & ((1ull << lane) - 1));
        nextd += lane == dd ? (uint32_t)__popcll(m) : 0u;
      }
      if (i < asize) code[i] = d ? (uint16_t)(__brev(v) >> (32 - d)) : (uint16_t)0;
    }
    wave_sync();
  }
  {
    BitW w{buf, 0};
    if (n > 4) {   // the complex form (the codes are assigned above)
      store_complex_wave(w, depth, asize, ts, reinterpret_cast<uint32_t *>(buf), &sh_nr);
    } else if (lane == 0) {
      store_code(w, n, nzs, max_bits, depth, code, asize, ts, n > 1);
    }
    if (lane == 0) {
      w.flush();
      mb.tree_bits[t] = (uint32_t)w.pos;
    }
  }
#ifdef MIB_PROF
  if (lane == 0) {
    const uint64_t te = HPT();
    atomicAdd(&g_huff_prof[0], 1ull);
    atomicAdd(&g_huff_prof[1], (unsigned long long)hp_att);
    atomicAdd(&g_huff_prof[2], (unsigned long long)hp_sort);
    atomicAdd(&g_huff_prof[3], (unsigned long long)hp_tree);
    atomicAdd(&g_huff_prof[4], (unsigned long long)(te - tc));
    atomicAdd(&g_huff_prof[5], (unsigned long long)(te - hp0));
    atomicAdd(&g_huff_prof[6], (unsigned long long)n);
    if (hp_att > 1) atomicAdd(&g_huff_prof[7], 1ull);
    atomicMax(&g_huff_prof[8], (unsigned long long)(te - hp0));
    atomicMax(&g_huff_prof[9], (unsigned long long)hp_sort);
    atomicMax(&g_huff_prof[10], (unsigned long long)hp_tree);
    atomicMax(&g_huff_prof[11], (unsigned long long)(te - tc));
  }
#endif
  wave_sync();
  uint8_t *dst = trees + ((size_t)m * kTreeSlots + t) * kTreeBytes;
  for (int i = lane; i < kTreeBytes; i += 64) dst[i] = buf[i];
  Codes &cd = codes[m];
  uint8_t *dd = lit ? cd.ld[cl] : !dist ? cd.cd[cl] : cd.dd[cl];
  uint16_t *cc = lit ? cd.lc[cl] : !dist ? cd.cc[cl] : cd.dcd[cl];
  for (int i = lane; i < asize; i += 64) {
    dd[i] = depth[i];
    cc[i] = code[i];
  }
  };
  item(t0);
  if (t1 >= 0) {
    wave_sync();
    item(t1);
  }
}


// ---------------------------------------------------------------- block split: block per (metablock, category)
// splitByteVector / findBlocks / clusterBlocks (block-splitter.ts:117-464) restated over
// block-split units (8 KiB of commands) instead of single symbols: kMaxBT block types are
// seeded as contiguous runs of units, then refined kSplitIters times -- type histograms,
// per-symbol bit costs (log2 total - log2 count, block-splitter.ts:150-160), each unit's cost
// under every type, and a shortest path over the units with the reference's block switch
// cost (26.0 bits literals, 28.1 commands / distances, :431-459).  The split is kept when it
// beats one block type by more than its header cost.  Types are renumbered by first use (the
// first block is type 0), then the block switches are laid out: each switch sits before the
// first symbol of its unit and carries the type code (second-to-last / last + 1 / explicit,
// RFC 7932 section 6) and the count of the new block; the block type and count prefix codes
// are built here (serial, <= 26 symbols).
constexpr int kMaxUnits = (int)(kMaxMetablock >> kSubBits);
constexpr int kSplitIters = 4;
constexpr int kPathCL = 16;        // units per chunk of the split's shortest path (at least)
constexpr int kPathChunks = 128;   // chunks at most (scratch in th: 128 x (16 + 4) floats + 4 x 128 bytes)
__device__ __forceinline__ float sym_bits(uint32_t c, float log_total) {
  return c ? log_total - __log2f((float)c) : log_total + 2.f;
}
// NT threads per (metablock, category) block: 1024 when the blocks do not fill the chip (one
// long stream: its few metablocks), else 256; the type histograms sum NT / 256 unit ranges in
// parallel, every float sum keeps the 256-thread grouping (identical output either way)
#ifdef MIB_PROF   // timing experiment: cycles per phase of the split (thread 0's view)
__device__ unsigned long long g_split_prof[8];
#define SPMARK(k)                                       \
  do {                                                  \
    if (t == 0) {                                       \
      const uint64_t t_ = __builtin_amdgcn_s_memtime(); \
      sp[k] += t_ - sp0;                                \
      sp0 = t_;                                         \
    }                                                   \
  } while (0)
#else
#define SPMARK(k) do {} while (0)
#endif
// Exclusive scans of two per-unit series fa(i), fb(i) over i < n into ea / eb (eb may be null),
// a thread per run of ceil(n / NT) units, the runs' sums scanned in LDS (wa, wb: NT each);
// every thread gets the totals.  Ends with a barrier.
template <int NT, class FA, class FB>
__device__ void block_scan2(int t, int n, FA fa, FB fb, uint32_t *ea, uint32_t *eb, uint32_t *wa, uint32_t *wb, uint32_t &ta,
                            uint32_t &tb) {
  const int per = (n + NT - 1) / NT, lo = min(n, t * per), hi = min(n, lo + per);
  uint32_t sa = 0, sb = 0;
  for (int i = lo; i < hi; i++) {
    sa += fa(i);
    sb += fb(i);
  }
  wa[t] = sa;
  wb[t] = sb;
  __syncthreads();
  for (int o = 1; o < NT; o <<= 1) {
    const uint32_t va = t >= o ? wa[t - o] : 0u, vb = t >= o ? wb[t - o] : 0u;
    __syncthreads();
    wa[t] += va;
    wb[t] += vb;
    __syncthreads();
  }
  uint32_t xa = wa[t] - sa, xb = wb[t] - sb;
  for (int i = lo; i < hi; i++) {
    ea[i] = xa;
    xa += fa(i);
    if (eb) eb[i] = xb;
    xb += fb(i);
  }
  ta = wa[NT - 1];
  tb = wb[NT - 1];
  __syncthreads();
}

// The split's shortest path with S states (S = 4 when the split seeds at most four types:
// the same sums as ever; else kMaxBT).  Scratch (in th): the
// chunks' S x S matrices, their start costs, exit maps (3 bits per state) and handed states.
// ucost rows are S wide.
template <int S, bool kLanes>
__device__ void split_path(int t, int nu, const uint32_t *ns, const float *ucost, uint8_t *asg, uint16_t *bp,
                           uint32_t *scratch, float sw_cost) {
  constexpr int kCh = S <= 4 ? kPathChunks : kPathChunks / 2;   // (the scratch fits th either way)
  static_assert(kCh * (S * S + S) * 4 + kCh * 7 <= S * 704 * 4, "path scratch fits th");
  const int CL = max(kPathCL, (nu + kCh - 1) / kCh);
  const int nch = (nu + CL - 1) / CL;
  float *Tm = reinterpret_cast<float *>(scratch);   // [nch][S * S]: (q, p) -> cost
  float *Sd = Tm + kCh * S * S;                     // [nch][S]: costs at the chunk start
  uint32_t *Xm = reinterpret_cast<uint32_t *>(Sd + kCh * S);   // exit maps
  uint8_t *Pc = reinterpret_cast<uint8_t *>(Xm + kCh), *Qp = Pc + kCh, *Ln = Qp + kCh;
  constexpr float kBig = 1e30f;
  {   // the chunks' transfer matrices: a lane per entry (q, p) = lane S q + p of a chunk's S x S
      // lanes (64 / S^2 chunks a wave); a column's minimum over q by xor shuffles (a minimum is
      // exact in any order, so the entries are the serial walk's bit for bit).  (A thread per
      // chunk took S^2 steps a unit: the cadence's 1 MiB metablocks have 8 chunks of 16 units.)
    constexpr int kE = S * S, kPer = 64 / kE;   // lanes a chunk, chunks a wave
    const int lane = t & 63, e = lane % kE, q = e / S;
    const int nwv = (int)(blockDim.x >> 6);
    for (int c0 = (t >> 6) * kPer; c0 < nch; c0 += nwv * kPer) {
      const int c = c0 + lane / kE;   // this lane's chunk (past nch: idle lanes, same steps)
      float T = (e / S) == (e % S) ? 0.f : kBig;
      const int ib = c * CL, i1 = min(nu, ib + CL);
      for (int k = 0; k < CL; k++) {
        const int i = ib + k;
        const bool live = c < nch && i < i1 && ns[i] != 0u;
        float col = T;
#pragma unroll
        for (int o = S; o < kE; o <<= 1) col = fminf(col, __shfl_xor(col, o, 64));
        col += sw_cost;
        const float u = live ? ucost[i * S + q] : 0.f;
        T = live ? fminf(T, col) + u : T;
      }
      if (c < nch) Tm[c * kE + e] = T;
    }
  }
  __syncthreads();
  if (t == 0) {   // the costs at every chunk start
    float dp[S];
#pragma unroll
    for (int q = 0; q < S; q++) dp[q] = 0.f;
    for (int c = 0; c < nch; c++) {
      float nd[S];
#pragma unroll
      for (int q = 0; q < S; q++) {
        Sd[c * S + q] = dp[q];
        float v = kBig;
#pragma unroll
        for (int p = 0; p < S; p++) v = fminf(v, Tm[c * S * S + S * q + p] + dp[p]);
        nd[q] = v;
      }
#pragma unroll
      for (int q = 0; q < S; q++) dp[q] = nd[q];
    }
    int cur = 0;
    for (int q = 1; q < S; q++)
      if (dp[q] < dp[cur]) cur = q;
    Pc[kCh - 1] = (uint8_t)cur;   // (handed to the last chunk below)
  }
  __syncthreads();
  if constexpr (kLanes) {   // replay: the serial walk's switch bits, then the chunk's exit map -- a lane per state q
      // of a chunk's S lanes (64 / S chunks a wave).  The unit's best state is the group's
      // minimum (exact in any order) and, as the serial scan's strict '<' picks, the lowest q
      // holding it below 1e30; the exit map walks back a lane per entry state.
    constexpr int kPer = 64 / S;
    const int lane = t & 63, q = lane % S, g = lane / S;
    const uint64_t gmask = (S == 64 ? ~0ull : ((1ull << S) - 1)) << (g * S);
    const int nwv = (int)(blockDim.x >> 6);
    for (int c0 = (t >> 6) * kPer; c0 < nch; c0 += nwv * kPer) {
      const int c = c0 + g;   // (past nch: idle lanes, same steps)
      const int i0 = c * CL, i1 = min(nu, i0 + CL);
      float dq = c < nch ? Sd[c * S + q] : 0.f;
      for (int k = 0; k < CL; k++) {
        const int i = i0 + k;
        const bool live = c < nch && i < i1 && ns[i] != 0u;
        float m = dq;
#pragma unroll
        for (int o = 1; o < S; o <<= 1) m = fminf(m, __shfl_xor(m, o, 64));
        const float best = fminf(m, 1e30f);
        const uint64_t eq = __ballot(dq == best && dq < 1e30f) & gmask;
        const int bq = eq ? (__ffsll((unsigned long long)(eq >> (g * S))) - 1) : 0;
        const float sw = best + sw_cost;
        const bool sv = sw < dq;   // (never at the first unit: every cost is 0 there)
        const uint32_t bb = (uint32_t)((__ballot(sv) & gmask) >> (g * S));
        const float nd = (sv ? sw : dq) + (live ? ucost[i * S + q] : 0.f);
        if (live && q == 0) bp[i] = (uint16_t)(bb | (uint32_t)(bq << 8));
        dq = live ? nd : dq;
      }
      wave_sync();   // (bp of this wave's chunks, written by their lanes q = 0)
      int cur = q;
      for (int i = i1 - 1; i >= i0; i--)
        if (c < nch && ns[i] && (bp[i] >> cur & 1)) cur = bp[i] >> 8;
      uint32_t xm = (uint32_t)cur << (3 * q);
#pragma unroll
      for (int o = 1; o < S; o <<= 1) xm |= (uint32_t)__shfl_xor((int)xm, o, 64);
      if (c < nch && q == 0) Xm[c] = xm;
    }
  } else if (t < nch) {   // (a thread per chunk: the batch build, whose registers the lane form raised past three waves a SIMD, C4 -0.8 %)
    float dp[S];
#pragma unroll
    for (int q = 0; q < S; q++) dp[q] = Sd[t * S + q];
    const int i0 = t * CL, i1 = min(nu, (t + 1) * CL);
    for (int i = i0; i < i1; i++) {
      if (!ns[i]) continue;
      float best = 1e30f;
      int bq = 0;
#pragma unroll
      for (int q = 0; q < S; q++)
        if (dp[q] < best) {
          best = dp[q];
          bq = q;
        }
      uint32_t bb = 0;
      float nd[S];
#pragma unroll
      for (int q = 0; q < S; q++) {
        const float stay = dp[q], sw = best + sw_cost;
        const bool sv = sw < stay;   // (never at the first unit: every cost is 0 there)
        nd[q] = (sv ? sw : stay) + ucost[i * S + q];
        if (sv) bb |= 1u << q;
      }
      bp[i] = (uint16_t)(bb | (uint32_t)(bq << 8));
#pragma unroll
      for (int q = 0; q < S; q++) dp[q] = nd[q];
    }
    uint32_t xm = 0;
    for (int cin = 0; cin < S; cin++) {
      int cur = cin;
      for (int i = i1 - 1; i >= i0; i--)
        if (ns[i] && (bp[i] >> cur & 1)) cur = bp[i] >> 8;
      xm |= (uint32_t)cur << (3 * cin);
    }
    Xm[t] = xm;
  }
  __syncthreads();
  if (t == 0) {   // the state handed into every chunk from the right
    int cur = Pc[kCh - 1];
    for (int c = nch - 1; c >= 0; c--) {
      Pc[c] = (uint8_t)cur;
      cur = (int)((Xm[c] >> (3 * cur)) & 7);
    }
  }
  __syncthreads();
  if (t < nch) {   // the chunk's assignment; its last non-empty unit's type
    int cur = Pc[t], ln = -1;
    const int i0 = t * CL, i1 = min(nu, (t + 1) * CL);
    for (int i = i1 - 1; i >= i0; i--) {
      if (!ns[i]) continue;
      asg[i] = (uint8_t)cur;
      if (ln < 0) ln = cur;
      if (bp[i] >> cur & 1) cur = bp[i] >> 8;
    }
    Ln[t] = (uint8_t)(ln < 0 ? 0xFF : ln);
  }
  __syncthreads();
  if (t == 0) {   // empty units follow their predecessor: the type handed into each chunk
    int prev = asg[0];
    for (int c = 0; c < nch; c++) {
      Qp[c] = (uint8_t)prev;
      if (Ln[c] != 0xFF) prev = Ln[c];
    }
  }
  __syncthreads();
  if (t < nch) {
    int prev = Qp[t];
    const int i0 = t * CL, i1 = min(nu, (t + 1) * CL);
    for (int i = i0; i < i1; i++) {
      if (!ns[i]) asg[i] = (uint8_t)prev;
      prev = asg[i];
    }
  }
}

// The block types a split may seed per category (literal, command, distance): the split is
// tried with K types; types the shortest path leaves unused drop out.  Literals take up to 8
// (C4 0.36469 -> 0.36365 compressed, C3 0.45579 -> 0.45569, decode unchanged; r04ad / r04ae).  Commands and distances keep 4:
// with 8 their prefix codes overflow the decoder's LDS table area (§7) and C4 decode goes from
// 140 to 299 ms for 0.05 % of bytes.  (A/B: MIB_SPLIT_BT = "l,c,d", each 1..kMaxBT.)
constexpr int kSplitBtLit = 8;
constexpr float kExtraTypeBits = 400.f;
// a four-type command / distance split that saved at least this share of the one-type cost is
// tried again with eight seeds (the heterogeneous input of test_more_than_four_command_and_
// distance_block_types: 0.217 for commands; C4's text ~0.010 / 0.035, C3's glyphs 0.05-0.09,
// r06k): past four types the data must differ in kind
constexpr float kWidenGain = 0.15f;   // a literal code's worth (C4: 24 -> 16 literal codes, +0.1 % bytes, r06d)
__device__ __forceinline__ int nu_of(const Mb &mb) { return (int)mb.nseg * kSubPerSeg; }
struct SplitK { int k[3]; int dbg; int widen; };
SplitK split_k() {
  static const SplitK sk = [] {
    SplitK k{{kSplitBtLit, 4, 4}, 0, 0};
    if (const char *e = knob("MIB_SPLIT_BT")) sscanf(e, "%d,%d,%d", &k.k[0], &k.k[1], &k.k[2]);
    k.dbg = knob("MIB_SPLIT_PRINT") ? atoi(knob("MIB_SPLIT_PRINT")) : 0;   // (experiments: the first n metablocks' split costs)
    for (int c = 0; c < 3; c++) k.k[c] = std::min(kMaxBT, std::max(1, k.k[c]));
    return k;
  }();
  return sk;
}
// S: the refinement's states (4, or kMaxBT): a launch per S, each taking the (metablock,
// category) blocks whose K it covers (K <= 4: S = 4, the loops and LDS of four types)
template <int NT, int S>
__global__ __launch_bounds__(NT) void split_kernel(const Job *jobs, Mb *mbs, int nmbs, Unit *units, const uint32_t *unit_h,
                                                    Codes *codes, SplitK sk) {
  __shared__ uint32_t th[S][704];
  __shared__ float bc[S][704];
  extern __shared__ float ucost[];   // [units][S] (launch_split sizes it for the largest metablock)
  __shared__ uint8_t asg[kMaxUnits];
  __shared__ uint16_t bp[kMaxUnits];   // switch bits per state | best state << 8
  __shared__ uint32_t ns[kMaxUnits];   // the units' symbol counts (the serial steps read them from LDS)
  __shared__ uint32_t tot[S];
  constexpr int kSplitT = NT;
  __shared__ float red[kSplitT];
  __shared__ uint32_t scan_b[kSplitT];   // (block scans: red and this hold the threads' partial sums)
  __shared__ int sh_ne, sh_keep;
  const int m = blockIdx.x / 3, cat = blockIdx.x % 3;
  Mb &mb = mbs[m];
  const Job &jb = jobs[mb.job];
  if (jb.uncompressed) return;
  const int t = threadIdx.x;
  // (literals: the metablock's 24 codes -- the decoder's LDS budget -- serve more block types
  // in a short metablock, more contexts per type in a long one; FONT mode keeps 4: C3 0.45579
  // -> 0.45569 for 2 % of its MB/s, r04am)
  int K = cat == 0 && (nu_of(mbs[m]) > kSplitWideUnits || jobs[mbs[m].job].font) ? min(sk.k[0], 4) : sk.k[cat];
  if (sk.widen) {
    // the widening pass (launch_split): command / distance categories whose four-type split
    // saved at least kWidenGain of the one-type cost are split again with kMaxBT seeds
    if constexpr (S == 4) return;
    if (cat == 0 || K > 4 || !(mb.split_gain[cat] >= kWidenGain)) return;
    K = kMaxBT;
  } else if ((K <= 4) != (S == 4)) {
    return;   // (the other launch's block)
  }
#ifdef MIB_PROF
  uint64_t sp[8] = {0, 0, 0, 0, 0, 0, 0, 0}, sp0 = __builtin_amdgcn_s_memtime();
#endif
  const int A = cat == 0 ? 256 : cat == 1 ? 704 : 16 + (int)jb.ndirect + (48 << jb.npostfix);
  const int hoff = cat == 0 ? 0 : cat == 1 ? 256 : 256 + 704;
  const float sw_cost = cat == 0 ? 26.0f : 28.1f;
  const uint32_t u0 = mb.first_seg * kSubPerSeg;
  const int nu = (int)mb.nseg * kSubPerSeg;
  Unit *U = units + u0;
  const uint32_t *H = unit_h + (size_t)u0 * kSubHist + hoff;
  for (int i = t; i < nu; i += kSplitT) ns[i] = U[i].nsym[cat];
  __syncthreads();
  SPMARK(0);
  // seed: the non-empty units in K contiguous runs (unit i: rank r among them, type r K / ne)
  {
    uint32_t *rk = &th[0][0];
    uint32_t nne, unused;
    block_scan2<NT>(t, nu, [&](int i) -> uint32_t { return ns[i] ? 1u : 0u; }, [&](int) -> uint32_t { return 0u; }, rk,
                    static_cast<uint32_t *>(nullptr), reinterpret_cast<uint32_t *>(red), scan_b, nne, unused);
    for (int i = t; i < nu; i += kSplitT) asg[i] = (uint8_t)(nne ? (rk[i] * (uint32_t)K) / nne : 0u);
    if (t == 0) sh_ne = (int)nne;
    __syncthreads();
  }
  SPMARK(1);
  const int ne = sh_ne;
  int keep = 0;
  // the refinement: S-wide loops and unit-cost rows
  auto refine = [&]() -> int {
    float base_cost = 0.f;
    constexpr int kRowK = (704 + 63) / 64;
    const int lx = t & 63;
    auto load_row = [&](int i, uint32_t (&v)[kRowK]) {
      const uint32_t *h = H + (size_t)i * kSubHist;
#pragma unroll
      for (int k = 0; k < kRowK; k++) v[k] = (i < nu && ns[i] && lx + 64 * k < A) ? h[lx + 64 * k] : 0u;
    };
    for (int it = 0; it <= kSplitIters; it++) {
      // type histograms (it == kSplitIters: of the final assignment); one type = all units.
      // NT / 256 unit ranges in parallel (256 symbols each), summed with LDS atomics
      for (int x = t; x < A; x += kSplitT)
        for (int q = 0; q < S; q++) th[q][x] = 0;
      __syncthreads();
      {
        // a thread per (unit range, four symbols): 16-byte row loads, eight rows a batch issued
        // together (a load-use pair per row left one HBM/L2 round trip per row in flight; 4-byte
        // loads kept the block's few waves waiting on the latency: C2's 16 MiB metablocks read
        // each 704-wide command row 2,048 times an iteration)
        constexpr int kV = S <= 4 ? 4 : 2;   // symbols a thread (registers: kV x S sums)
        typedef typename std::conditional<kV == 4, uint4, uint2>::type VT;
        auto vget = [](const VT &v, int k) -> uint32_t {
          if constexpr (kV == 4) return k == 0 ? v.x : k == 1 ? v.y : k == 2 ? v.z : v.w;
          else return k == 0 ? v.x : v.y;
        };
        const int ng = (A + kV - 1) / kV, nr = max(1, kSplitT / ng);
        const int qd = t / ng, g = t % ng;
        if (qd < nr) {
          const int i0 = (nu * qd) / nr, i1 = (nu * (qd + 1)) / nr;
          uint32_t s[kV][S];
#pragma unroll
          for (int k = 0; k < kV; k++)
#pragma unroll
            for (int q = 0; q < S; q++) s[k][q] = 0;
          const VT *hrow = reinterpret_cast<const VT *>(H + kV * g);   // (rows and the category's offset are 16-byte aligned)
          constexpr uint32_t kRowV = kSubHist / kV;
          int i = i0;
          for (; i + 8 <= i1; i += 8) {
            VT v[8];
#pragma unroll
            for (int j = 0; j < 8; j++) v[j] = hrow[(size_t)(i + j) * kRowV];
#pragma unroll
            for (int j = 0; j < 8; j++) {
              const int a = asg[i + j];
#pragma unroll
              for (int k = 0; k < kV; k++)
#pragma unroll
                for (int q = 0; q < S; q++) s[k][q] += a == q ? vget(v[j], k) : 0u;
            }
          }
          for (; i < i1; i++) {
            const VT v = hrow[(size_t)i * kRowV];
            const int a = asg[i];
#pragma unroll
            for (int k = 0; k < kV; k++)
#pragma unroll
              for (int q = 0; q < S; q++) s[k][q] += a == q ? vget(v, k) : 0u;
          }
#pragma unroll
          for (int k = 0; k < kV; k++)
            if (kV * g + k < A)
#pragma unroll
              for (int q = 0; q < S; q++)
                if (s[k][q]) atomicAdd(&th[q][kV * g + k], s[k][q]);
        }
      }
      __syncthreads();
      SPMARK(2);
      if (t < S) {
        uint32_t s = 0;
        for (int x = 0; x < A; x++) s += th[t][x];
        tot[t] = s;
      }
      __syncthreads();
      if (it == 0) {   // the one-type baseline: entropy of the merged histogram + one code's header
        float part = 0.f;
        uint32_t all = 0;
        for (int q = 0; q < S; q++) all += tot[q];
        const float la = __log2f((float)all);
        int nz = 0;
        for (int x = t; t < 256 && x < A; x += 256) {
          uint32_t c = 0;
          for (int q = 0; q < S; q++) c += th[q][x];
          if (c) {
            part += (float)c * (la - __log2f((float)c));
            nz++;
          }
        }
        red[t] = part + 3.5f * (float)nz;
        __syncthreads();
        for (int o = kSplitT / 2; o; o >>= 1) {
          if (t < o) red[t] += red[t + o];
          __syncthreads();
        }
        base_cost = red[0] + 40.f;
        __syncthreads();
      }
      for (int x = t; x < A; x += kSplitT)
        for (int q = 0; q < S; q++) bc[q][x] = tot[q] ? sym_bits(th[q][x], __log2f((float)tot[q])) : 1e9f;
      __syncthreads();
      SPMARK(3);
      if (it == kSplitIters) break;
      // every unit's bits under every type: a wave per unit, lanes over the symbols
      // (the unit's row is loaded whole, one unit ahead -- up to 22 loads a lane in flight; the
      // sums in the same order as ever)
      uint32_t rv[kRowK], rn[kRowK];
      load_row(t >> 6, rv);
      for (int i = t >> 6; i < nu; i += kSplitT / 64) {
        load_row(i + kSplitT / 64, rn);   // the wave's next unit, in flight while this one is summed
        float c[S];
#pragma unroll
        for (int q = 0; q < S; q++) c[q] = 0.f;
        if (ns[i]) {
#pragma unroll
          for (int k = 0; k < kRowK; k++) {
            const int x = lx + 64 * k;
            if (x < A) {
              const float v = (float)rv[k];
#pragma unroll
              for (int q = 0; q < S; q++) c[q] += v * bc[q][x];
            }
          }
#pragma unroll
          for (int q = 0; q < S; q++)
            for (int o = 32; o; o >>= 1) c[q] += __shfl_xor(c[q], o);
        }
        if (lx == 0)
          for (int q = 0; q < S; q++) ucost[i * S + q] = q < K ? c[q] : 1e30f;   // (types past K: empty)
#pragma unroll
        for (int k = 0; k < kRowK; k++) rv[k] = rn[k];
      }
      __syncthreads();
      SPMARK(4);
      // shortest path over the non-empty units with the switch cost (findBlocks' DP), in
      // chunks of kPathCL units so that it is not one thread's serial walk (2,048 units of a
      // 16 MiB metablock: 6.3 M cycles, most of the kernel).  A unit maps the costs of the four
      // states to dp'[q] = min(dp[q], min dp + switch) + ucost[q], a (min, +) product: each
      // chunk composes its units' 4 x 4 matrices, one thread carries the costs across the
      // chunks, each chunk then replays its units from its start costs as the serial walk does
      // (the switch bits), and the backtrack runs per chunk from the state handed in from
      // the right (one thread chains the chunks' exit maps).  Scratch: th, which the next
      // iteration recomputes.
      split_path<S, NT == 1024>(t, nu, ns, ucost, asg, bp, &th[0][0], sw_cost);
      __syncthreads();
      SPMARK(5);
    }
    // the split's cost: unit bits under the final histograms, switches, one code header per type
    float part = 0.f;   // (the first 256 threads, in the same grouping as ever: identical sums)
    if (t < 256) {
      uint32_t fv[kRowK], fn[kRowK];
      load_row(t >> 6, fv);
      for (int i = t >> 6; i < nu; i += 4) {
        load_row(i + 4, fn);
        if (ns[i]) {
          const int q = asg[i];
#pragma unroll
          for (int k = 0; k < kRowK; k++)
            if (lx + 64 * k < A) part += (float)fv[k] * bc[q][lx + 64 * k];
        }
#pragma unroll
        for (int k = 0; k < kRowK; k++) fv[k] = fn[k];
      }
    }
    for (int x = t; t < 256 && x < A; x += 256)
      for (int q = 0; q < S; q++) part += th[q][x] ? 3.5f : 0.f;
    red[t] = part;
    __syncthreads();
    for (int o = kSplitT / 2; o; o >>= 1) {
      if (t < o) red[t] += red[t + o];
      __syncthreads();
    }
    if (t == 0) {
      int nsw = 0, used = 0, prev = -1;
      for (int i = 0; i < nu; i++) {
        if (!ns[i]) continue;
        if (prev >= 0 && asg[i] != prev) nsw++;
        prev = asg[i];
      }
      for (int q = 0; q < S; q++) used += tot[q] ? 1 : 0;
      const float split_cost = red[0] + 40.f * (float)used + sw_cost * (float)nsw + 60.f;
      sh_keep = (used > 1 && split_cost < base_cost) ? 1 : 0;
      if (!sk.widen) mb.split_gain[cat] = sh_keep ? (base_cost - split_cost) / base_cost : 0.f;
      if (m < sk.dbg) printf("[split] mb %d cat %d K %d used %d units %d base %.0f split %.0f gain %.4f\n", m, cat, K, used, ne,
                             base_cost, split_cost, (base_cost - split_cost) / base_cost);
    }
    __syncthreads();
    SPMARK(6);
    return sh_keep;
  };
  if (K > 1 && ne >= 2 * K) keep = refine();
  else if (t == 0 && !sk.widen) mb.split_gain[cat] = 0.f;
  if constexpr (S > 4) {
    // Command / distance types past four (the reference allows 256) take room from
    // the literal codes in the decoder's LDS table area (cluster_kernel's budget: two literal
    // codes a command type, four a distance type).  So past four types, the two types whose
    // merge costs the fewest bits merge while that is less than what the extra type displaces
    // (kExtraTypeBits): homogeneous data (C4's text) keeps four or fewer, a metablock whose
    // units differ in kind keeps more.
    if (keep && cat > 0) {
      __shared__ float pair_d[kMaxBT * (kMaxBT - 1) / 2];
      __shared__ int sh_merge;
      const float penalty = cat == 1 ? kExtraTypeBits * 2.f : kExtraTypeBits * 4.f;
      for (;;) {
        int used = 0;
        for (int q = 0; q < S; q++) used += tot[q] ? 1 : 0;
        if (used <= 4) break;
        // thread per type pair: the bits the merge adds (entropy, 3.5 bits a used symbol, one
        // code header of 40 bits fewer)
        if (t < S * (S - 1) / 2) {
          int a = 0, r = t;
          while (r >= S - 1 - a) {
            r -= S - 1 - a;
            a++;
          }
          const int b = a + 1 + r;
          float d = 1e30f;
          if (tot[a] && tot[b]) {
            const float la = __log2f((float)tot[a]), lb = __log2f((float)tot[b]), lab = __log2f((float)(tot[a] + tot[b]));
            float e = -40.f;
            for (int x = 0; x < A; x++) {
              const uint32_t ca = th[a][x], cb = th[b][x];
              if (!(ca | cb)) continue;
              const float cab = (float)(ca + cb);
              e += cab * (lab - __log2f(cab)) + 3.5f;
              if (ca) e -= (float)ca * (la - __log2f((float)ca)) + 3.5f;
              if (cb) e -= (float)cb * (lb - __log2f((float)cb)) + 3.5f;
            }
            d = e;
          }
          pair_d[t] = d;
        }
        __syncthreads();
        if (t == 0) {
          int bi = 0;
          for (int k2 = 1; k2 < S * (S - 1) / 2; k2++)
            if (pair_d[k2] < pair_d[bi]) bi = k2;
          sh_merge = pair_d[bi] < penalty ? bi : -1;
        }
        __syncthreads();
        if (sh_merge < 0) break;
        int a = 0, r = sh_merge;
        while (r >= S - 1 - a) {
          r -= S - 1 - a;
          a++;
        }
        const int b = a + 1 + r;
        for (int i = t; i < nu; i += kSplitT)
          if (asg[i] == b) asg[i] = (uint8_t)a;
        for (int x = t; x < A; x += kSplitT) {
          th[a][x] += th[b][x];
          th[b][x] = 0;
        }
        __syncthreads();
        if (t == 0) {
          tot[a] += tot[b];
          tot[b] = 0;
        }
        __syncthreads();
      }
    }
  }
#ifdef MIB_PROF
  const uint64_t tail0 = __builtin_amdgcn_s_memtime();
#endif
  if (!keep) {
    for (int i = t; i < nu; i += kSplitT) {
      U[i].type[cat] = 0;
      U[i].sw_count[cat] = 0;
    }
    if (t == 0) {
      mb.nbt[cat] = 1;
      mb.first_count[cat] = 0;
    }
    return;
  }
  // The layout works in LDS (the unit costs, switch bits and histograms are dead here): per
  // unit its type, the count of the block a switch there opens, the switch's code; the units
  // are then written by every thread.  In parallel (a serial walk by one thread was ~800
  // cycles a unit, 20 % of the kernel on 16 MiB metablocks): types renumbered by first use;
  // a switch wherever a non-empty unit's type differs from the one before it (an empty unit
  // carries its predecessor's type); scans give each switch its rank and each unit the
  // symbols before it, so block b's count and its code (from the two blocks before it,
  // RFC 7932 section 6) need no walk.
  uint32_t *lsw = reinterpret_cast<uint32_t *>(ucost);                      // [nu]
  uint8_t *lcode = reinterpret_cast<uint8_t *>(lsw + nu);                   // [nu]
  uint32_t *swu = reinterpret_cast<uint32_t *>(lcode + ((nu + 3) & ~3));    // [nu]: unit of switch k
  uint8_t *btype = reinterpret_cast<uint8_t *>(swu + nu);                   // [nu + 1]: type of block b
  static_assert(kSubPerSeg >= 4, "10 bytes a unit + 4 fit the unit costs' 16");
  uint32_t *cum = &th[0][0];                                                // [nu + 1]: symbols before unit i
  uint32_t *swr = reinterpret_cast<uint32_t *>(&bc[0][0]);                  // [nu]: switches before unit i
  static_assert(4 * 704 >= kMaxUnits + 1, "th / bc hold a value per unit");
  uint8_t *lty = reinterpret_cast<uint8_t *>(bp);
  __shared__ int sh_first[kMaxBT + 1];   // first non-empty unit of each type; [kMaxBT]: of any
  __shared__ uint8_t sh_map[kMaxBT];
  __shared__ uint32_t sh_hcode[kMaxBT + 2], sh_hcount[26];
  if (t <= kMaxBT) sh_first[t] = 0x7FFFFFFF;
  if (t < kMaxBT + 2) sh_hcode[t] = 0;
  if (t < 26) sh_hcount[t] = 0;
  __syncthreads();
  for (int i = t; i < nu; i += kSplitT)
    if (ns[i]) {
      atomicMin(&sh_first[asg[i]], i);
      atomicMin(&sh_first[kMaxBT], i);
    }
  __syncthreads();
  if (t == 0)
    for (int q = 0; q < S; q++) {
      int r = 0;
      for (int p = 0; p < S; p++) r += sh_first[p] < sh_first[q] ? 1 : 0;
      sh_map[q] = (uint8_t)r;
    }
  __syncthreads();
  int nt = 0;
  for (int q = 0; q < S; q++) nt += sh_first[q] != 0x7FFFFFFF ? 1 : 0;
  const int fne = sh_first[kMaxBT];
  auto is_sw = [&](int i) -> uint32_t { return (ns[i] && i > fne && asg[i] != asg[i - 1]) ? 1u : 0u; };
  for (int i = t; i < nu; i += kSplitT) {
    lty[i] = (uint8_t)(i < fne ? 0 : sh_map[asg[i]]);
    lsw[i] = 0;
  }
  uint32_t nsw, nsym;
  block_scan2<NT>(t, nu, is_sw, [&](int i) -> uint32_t { return ns[i]; }, swr, cum, reinterpret_cast<uint32_t *>(red),
                  scan_b, nsw, nsym);
  if (t == 0) {
    cum[nu] = nsym;
    btype[0] = 0;
  }
  for (int i = t; i < nu; i += kSplitT)
    if (is_sw(i)) {
      swu[swr[i]] = (uint32_t)i;
      btype[swr[i] + 1] = lty[i];
    }
  __syncthreads();
  for (int bl = t; bl <= (int)nsw; bl += kSplitT) {   // block bl: from switch bl - 1 (unit 0 for bl = 0) to the next
    const uint32_t st = bl == 0 ? 0u : swu[bl - 1], en = bl < (int)nsw ? swu[bl] : (uint32_t)nu;
    const uint32_t count = cum[en] - cum[st];
    atomicAdd(&sh_hcount[block_count_code(count)], 1u);
    if (bl == 0) {
      mb.first_count[cat] = count;
    } else {
      const int ty = btype[bl], last = btype[bl - 1], second = bl >= 2 ? btype[bl - 2] : 1;
      const int code = ty == second ? 0 : ty == (last + 1) % nt ? 1 : ty + 2;
      lsw[st] = count;
      lcode[st] = (uint8_t)code;
      atomicAdd(&sh_hcode[code], 1u);
    }
  }
  __syncthreads();
  // the block-type and block-count codes by thread 0, every work array in LDS (as private
  // arrays indexed by data they lived in scratch memory: 1.7 KiB a lane, a global round trip
  // per access of the serial sort and tree walk)
  __shared__ SerialWs sws;
  __shared__ uint32_t sbl[16], snx[16];
  __shared__ uint8_t sdt[kMaxBT + 2], sdc[26];
  __shared__ uint16_t sct[kMaxBT + 2], scc[26];
  if (t == 0) {
    mb.nbt[cat] = (uint32_t)nt;
    serial_depths(sh_hcode, nt + 2, 15, sdt, sws);
    depths_to_codes(sdt, nt + 2, sct, sbl, snx);
    serial_depths(sh_hcount, 26, 15, sdc, sws);
    depths_to_codes(sdc, 26, scc, sbl, snx);
  }
  __syncthreads();
  {
    Codes &cd = codes[m];
    if (t < nt + 2) {
      cd.btd[cat][t] = sdt[t];
      cd.btc[cat][t] = sct[t];
    }
    if (t < 26) {
      cd.bcd[cat][t] = sdc[t];
      cd.bcc[cat][t] = scc[t];
    }
  }
  for (int i = t; i < nu; i += kSplitT) {
    Unit &u = U[i];
    u.type[cat] = lty[i];
    u.sw_count[cat] = lsw[i];
    if (lsw[i]) u.sw_code[cat] = lcode[i];
  }
#ifdef MIB_PROF
  if (t != 0) return;
  sp[7] += __builtin_amdgcn_s_memtime() - tail0;
  for (int q = 0; q < 8; q++) atomicAdd(&g_split_prof[q], (unsigned long long)sp[q]);
#endif
}

// encodeContextMap (context-map.ts:114-170): NTREES, then (NTREES > 1) move-to-front, runs
// of zeros as RLEMAX-prefixed run codes, a prefix code over NTREES + RLEMAX symbols, and the
// IMTF bit (RFC 7932 section 7.3).  Serial, one lane.
struct CmapWs {   // encode_context_map's work arrays (LDS)
  uint8_t mtf[kMaxLitTrees];
  uint8_t v[kLitSlots], sym[kLitSlots], nb[kLitSlots];
  uint16_t ex[kLitSlots];
  uint32_t hist[kMaxLitTrees + 16];
  uint8_t depth[kMaxLitTrees + 16];
  uint16_t code[kMaxLitTrees + 16];
  int16_t nzs[kMaxLitTrees + 16];
  SerialWs sw;
  TreeScratch ts;
};
// The move-to-front transform of a context map by the wave (all 64 lanes): lane l holds list
// entry l; per entry one ballot finds the value's place and one shuffle moves the ones before it
// back (~10 instructions, against ~10 dependent LDS round trips of the serial list walk).
__device__ void mtf_wave(const uint8_t *cmap, int size, uint8_t *v) {
  const int lane = threadIdx.x & 63;
  int m = lane;
  for (int i = 0; i < size; i++) {
    const int c = cmap[i];
    const uint64_t hit = __ballot(m == c);
    const int idx = __ffsll((unsigned long long)hit) - 1;
    if (lane == 0) v[i] = (uint8_t)idx;
    const int prev = __shfl_up(m, 1);
    m = lane == 0 ? c : lane <= idx ? prev : m;
  }
}
// (v: the context map's move-to-front values, mtf_wave)
__device__ void encode_context_map(BitW &w, const uint8_t *cmap, int size, int ntrees, CmapWs &ws) {
  put_varlen_u8(w, ntrees - 1);
  if (ntrees <= 1) return;
  uint8_t *v = ws.v, *sym = ws.sym, *nb = ws.nb, *depth = ws.depth;
  uint16_t *ex = ws.ex, *code = ws.code;
  uint32_t *hist = ws.hist;
  int16_t *nzs = ws.nzs;
  int maxrun = 0;
  for (int i = 0; i < size;) {
    int r = 0;
    while (i + r < size && v[i + r] == 0) r++;
    if (r > maxrun) maxrun = r;
    i += r ? r : 1;
  }
  int rlemax = 0;
  while ((2 << rlemax) <= maxrun && rlemax < 16) rlemax++;   // largest p with 2^p <= maxrun
  // symbols (code, extra bits, extra)
  int ns = 0;
  for (int i = 0; i < size;) {
    if (v[i] != 0) {
      sym[ns] = (uint8_t)(v[i] + rlemax);
      nb[ns] = 0;
      ex[ns++] = 0;
      i++;
      continue;
    }
    int L = 0;
    while (i + L < size && v[i + L] == 0) L++;
    i += L;
    while (L > 0) {
      if (L == 1 || rlemax == 0) {
        sym[ns] = 0;
        nb[ns] = 0;
        ex[ns++] = 0;
        L--;
        continue;
      }
      int p = 0;
      while ((2 << p) <= L && p < rlemax) p++;
      const int extra = min(L - (1 << p), (1 << p) - 1);
      sym[ns] = (uint8_t)p;
      nb[ns] = (uint8_t)p;
      ex[ns++] = (uint16_t)extra;
      L -= (1 << p) + extra;
    }
  }
  const int asize = ntrees + rlemax;
  for (int i = 0; i < asize; i++) hist[i] = 0;
  for (int k = 0; k < ns; k++) hist[sym[k]]++;
  w.put(1, rlemax > 0 ? 1 : 0);
  if (rlemax) w.put(4, (uint32_t)(rlemax - 1));
  int n = 0;
  for (int i = 0; i < asize; i++)
    if (hist[i]) nzs[n++] = (int16_t)i;
  serial_depths(hist, asize, 15, depth, ws.sw);
  int max_bits = 0;
  for (int c = asize - 1; c; c >>= 1) max_bits++;
  store_code(w, n, nzs, max_bits, depth, code, asize, ws.ts, false);
  for (int k = 0; k < ns; k++) {
    w.put(depth[sym[k]], code[sym[k]]);
    if (nb[k]) w.put(nb[k], ex[k]);
  }
  w.put(1, 1);   // IMTF
}

// encode_context_map by the wave (all 64 lanes call it; w is lane 0's writer): lane 0 forms the
// run-length symbols, the wave counts them, builds their code (serial_depths_wave) and writes
// them (wave_put_items) around lane 0's code header.  cnt2: two LDS ints.
__device__ void encode_context_map_wave(BitW &w, const uint8_t *cmap, int size, int ntrees, CmapWs &ws, uint32_t *buf32,
                                        int *cnt2) {
  const int lane = threadIdx.x & 63;
  if (lane == 0) put_varlen_u8(w, ntrees - 1);
  if (ntrees <= 1) return;
  uint8_t *v = ws.v, *sym = ws.sym, *nb = ws.nb, *depth = ws.depth;
  uint16_t *ex = ws.ex, *code = ws.code;
  uint32_t *hist = ws.hist;
  int16_t *nzs = ws.nzs;
  if (lane == 0) {
    int maxrun = 0;
    for (int i = 0; i < size;) {
      int r = 0;
      while (i + r < size && v[i + r] == 0) r++;
      if (r > maxrun) maxrun = r;
      i += r ? r : 1;
    }
    int rlemax = 0;
    while ((2 << rlemax) <= maxrun && rlemax < 16) rlemax++;   // largest p with 2^p <= maxrun
    int ns = 0;
    for (int i = 0; i < size;) {
      if (v[i] != 0) {
        sym[ns] = (uint8_t)(v[i] + rlemax);
        nb[ns] = 0;
        ex[ns++] = 0;
        i++;
        continue;
      }
      int L = 0;
      while (i + L < size && v[i + L] == 0) L++;
      i += L;
      while (L > 0) {
        if (L == 1 || rlemax == 0) {
          sym[ns] = 0;
          nb[ns] = 0;
          ex[ns++] = 0;
          L--;
          continue;
        }
        int p = 0;
        while ((2 << p) <= L && p < rlemax) p++;
        const int extra = min(L - (1 << p), (1 << p) - 1);
        sym[ns] = (uint8_t)p;
        nb[ns] = (uint8_t)p;
        ex[ns++] = (uint16_t)extra;
        L -= (1 << p) + extra;
      }
    }
    cnt2[0] = ns;
    cnt2[1] = rlemax;
  }
  wave_sync();
  const int ns = cnt2[0], rlemax = cnt2[1];
  const int asize = ntrees + rlemax;
  for (int i = lane; i < asize; i += 64) hist[i] = 0;
  wave_sync();
  for (int k = lane; k < ns; k += 64) atomicAdd(&hist[sym[k]], 1u);
  wave_sync();
  serial_depths_wave(hist, asize, 15, depth, ws.sw);
  if (lane == 0) {
    w.put(1, rlemax > 0 ? 1 : 0);
    if (rlemax) w.put(4, (uint32_t)(rlemax - 1));
    int n = 0;
    for (int i = 0; i < asize; i++)
      if (hist[i]) nzs[n++] = (int16_t)i;
    int max_bits = 0;
    for (int c = asize - 1; c; c >>= 1) max_bits++;
    store_code(w, n, nzs, max_bits, depth, code, asize, ws.ts, false);
    w.flush();
  }
  wave_sync();
  wave_put_items(w, buf32, ns, [&](int k, uint32_t &bits, uint32_t &val) {
    const int c = sym[k];
    const uint32_t d = depth[c];
    bits = d + nb[k];
    val = (uint32_t)code[c] | ((uint32_t)ex[k] << d);
  });
  if (lane == 0) w.put(1, 1);   // IMTF
}

// NBLTYPES and, for a split category, its block type and block count prefix codes and the
// first block count (storeBlockSwitch's header part, metablock.ts:150-220)
__device__ void put_block_split(BitW &w, int nbt, uint8_t *td, uint16_t *tc, uint8_t *cdp, uint16_t *cc, uint32_t first,
                                int16_t *nzs, TreeScratch &ts) {
  put_varlen_u8(w, nbt - 1);
  if (nbt <= 1) return;
  int n = 0;
  const int ta = nbt + 2;
  for (int i = 0; i < ta; i++)
    if (td[i]) nzs[n++] = (int16_t)i;
  int mb_bits = 0;
  for (int c = ta - 1; c; c >>= 1) mb_bits++;
  store_code(w, n, nzs, mb_bits, td, tc, ta, ts, false);
  n = 0;
  for (int i = 0; i < 26; i++)
    if (cdp[i]) nzs[n++] = (int16_t)i;
  store_code(w, n, nzs, 5, cdp, cc, 26, ts, false);
  const int bc = block_count_code(first);
  w.put(cdp[bc], cc[bc]);
  w.put((int)kBlkBits[bc], first - kBlkOff[bc]);
}

// The metablock header before the prefix codes (storeMetaBlock's header part,
// metablock.ts:690-705).  Block (one wave) per metablock: the header is written serially by
// lane 0 into LDS -- its bit writer's read-modify-write bytes and the context-map coder's work
// arrays were global / scratch memory round trips, 0.8 ms for a single metablock (a 1 MiB
// streaming chunk, r05m) -- then copied out by the wave.
__global__ __launch_bounds__(64) void mb_header_kernel(const Job *jobs, Mb *mbs, int nmbs, uint8_t *hdr, Codes *codes) {
  __shared__ __attribute__((aligned(16))) uint8_t hb[kHdrBytes];   // (words for the wave writers)
  __shared__ int sh_cm[2];
  __shared__ uint8_t map[kLitSlots];
  __shared__ int16_t nzs[26];
  __shared__ int sh_n, sh_ntrees;
  __shared__ CmapWs cws;
  __shared__ uint8_t btd[3][kMaxBT + 2], bcd[3][26];   // the block-split codes, staged by the wave
  __shared__ uint16_t btc[3][kMaxBT + 2], bcc[3][26];
  const int m = blockIdx.x;
  if (m >= nmbs) return;
  Mb &mb = mbs[m];
  const Job &jb = jobs[mb.job];
  if (jb.uncompressed) return;
  const int t = threadIdx.x;
  for (int i = t; i < kHdrBytes; i += 64) hb[i] = 0;
  {
    const Codes &cd = codes[m];
    for (int i = t; i < 3 * (kMaxBT + 2); i += 64) {
      btd[i / (kMaxBT + 2)][i % (kMaxBT + 2)] = cd.btd[i / (kMaxBT + 2)][i % (kMaxBT + 2)];
      btc[i / (kMaxBT + 2)][i % (kMaxBT + 2)] = cd.btc[i / (kMaxBT + 2)][i % (kMaxBT + 2)];
    }
    for (int i = t; i < 3 * 26; i += 64) {
      bcd[i / 26][i % 26] = cd.bcd[i / 26][i % 26];
      bcc[i / 26][i % 26] = cd.bcc[i / 26][i % 26];
    }
  }
  wave_sync();
  BitW w{hb, 0};   // (lane 0's)
  if (t == 0) {
    if (mb.start == 0 && jb.hdr_lgwin && !jb.parts) put_window_bits(w, (int)jb.hdr_lgwin);   // (else: part_index_kernel)
    const uint32_t length = mb.end - mb.start;
    w.put(1, mb.is_last);
    if (mb.is_last) w.put(1, 0);
    const int lg = length == 1 ? 1 : 32 - __clz(length - 1);
    const int mn = (lg < 16 ? 16 : lg + 3) / 4;
    w.put(2, (uint32_t)(mn - 4));
    w.put(mn * 4, length - 1);
    if (!mb.is_last) w.put(1, 0);
    for (int c = 0; c < 3; c++)
      put_block_split(w, (int)mb.nbt[c], btd[c], btc[c], bcd[c], bcc[c], mb.first_count[c], nzs, cws.ts);
    w.put(2, jb.npostfix);
    w.put(4, jb.ndirect >> jb.npostfix);
    for (uint32_t ty = 0; ty < mb.nbt[0]; ty++) w.put(2, mb.ctx_mode);
  }
  wave_sync();
  {   // store_code settles the codes it writes (a lone symbol's depth 0): back for the emitter
    Codes &cd = codes[m];
    for (int i = t; i < 3 * (kMaxBT + 2); i += 64) {
      cd.btd[i / (kMaxBT + 2)][i % (kMaxBT + 2)] = btd[i / (kMaxBT + 2)][i % (kMaxBT + 2)];
      cd.btc[i / (kMaxBT + 2)][i % (kMaxBT + 2)] = btc[i / (kMaxBT + 2)][i % (kMaxBT + 2)];
    }
    for (int i = t; i < 3 * 26; i += 64) {
      cd.bcd[i / 26][i % 26] = bcd[i / 26][i % 26];
      cd.bcc[i / 26][i % 26] = bcc[i / 26][i % 26];
    }
  }
  // the two context maps (literal, distance) over dense code indices: slots of type ty start at
  // the codes of the types before it; each map's move-to-front by the wave, its coding by lane 0
  for (int cat = 0; cat < 2; cat++) {
    const int nty = (int)(cat == 0 ? mb.nbt[0] : mb.nbt[2]), nctx = cat == 0 ? kLitCtx : kDistCtx;
    // (built by the wave from global memory: lane 0's loop of dependent loads took most of the
    // kernel's 0.36 ms, r05p)
    int base = 0, tbase = 0;   // codes of the types before mine / all types
    for (int ty = 0; ty < nty; ty++) {
      const int c = (int)(cat == 0 ? mb.nlit_t[ty] : mb.ndist_t[ty]);
      tbase += c;
    }
    for (int i = t; i < nty * nctx; i += 64) {
      const int ty = i / nctx;
      base = 0;
      for (int u = 0; u < ty; u++) base += (int)(cat == 0 ? mb.nlit_t[u] : mb.ndist_t[u]);
      map[i] = (uint8_t)(base + (cat == 0 ? mb.lit_cmap[i] - ty * kLitCtx : mb.dist_cmap[i] - ty * kDistCtx));
    }
    if (t == 0) {
      sh_n = nty * nctx;
      sh_ntrees = tbase;
    }
    wave_sync();
    if (sh_ntrees > 1) mtf_wave(map, sh_n, cws.v);
    wave_sync();
    encode_context_map_wave(w, map, sh_n, sh_ntrees, cws, reinterpret_cast<uint32_t *>(hb), sh_cm);
    wave_sync();
  }
  if (t == 0) {
    w.flush();
    mb.hdr_bits = (uint32_t)w.pos;
  }
  wave_sync();
  uint8_t *out = hdr + (size_t)m * kHdrBytes;
  for (int i = t; i < kHdrBytes; i += 64) out[i] = hb[i];
}

// ---------------------------------------------------------------- sizes: block per segment
// The segment's bit size: the sum of item_bits over its commands' items (the same
// load-balanced expansion as emit_kernel, so literal-heavy segments use every lane), kept per
// tile of kEmitTile commands too (tile_bits[segment][tile]: emit_kernel's tile offsets).
// Blocks per segment as emit_kernel's: block (s, y) sizes tiles y, y + gridDim.y, ... and adds
// its sum into the segment's bits (zero from the host's segment table).
template <int NT>
__global__ __launch_bounds__(NT) void sizes_kernel(const Job *jobs, Seg *segs, const Mb *mbs, const Cmd *cmds,
                                                       const uint32_t *cmd_pos, const Codes *codes, const Unit *units,
                                                       uint32_t *tile_bits) {
  static_assert(kEmitTile % NT == 0, "a tile is whole iterations");
  typedef hipcub::BlockScan<uint32_t, NT> Scan;
  typedef hipcub::BlockReduce<uint32_t, NT> Reduce;
  __shared__ typename Scan::TempStorage scan_tmp;
  __shared__ typename Reduce::TempStorage red_tmp;
  __shared__ ItemMap<NT> map;
  __shared__ Cmd sh_c[NT];
  __shared__ uint32_t sh_p[NT];
  __shared__ Unit sh_u[kSubPerSeg];
  Seg &sg = segs[blockIdx.x];
  const Job &jb = jobs[sg.job];
  if (jb.uncompressed) return;
  const uint32_t n = sg.ncmd + (sg.extra_ins ? 1 : 0);
  const uint32_t ntile = (n + kEmitTile - 1) / kEmitTile;
  if (blockIdx.y >= ntile) return;
  const int t = threadIdx.x;
  const Mb &mb = mbs[sg.mb];
  const Codes &cd = codes[sg.mb];
  __shared__ uint8_t sh_lut[512];   // per-literal lookups from LDS
  __shared__ uint16_t sh_cmap[kLitSlots];
  for (int i = t; i < 512; i += NT) sh_lut[i] = kRfcContextLut[(mb.ctx_mode << 9) + i];
  for (int i = t; i < kLitSlots; i += NT) sh_cmap[i] = mb.lit_cmap[i];
  if (t < kSubPerSeg) sh_u[t] = units[(size_t)blockIdx.x * kSubPerSeg + t];
  __syncthreads();
  const uint8_t *lut = sh_lut;
  uint32_t *tb = tile_bits + (size_t)blockIdx.x * kEmitTiles;
  unsigned long long total = 0;   // (thread 0)
  uint32_t tile = 0;              // (thread 0: the current tile's bits so far)
  for (uint32_t tl = blockIdx.y; tl < ntile; tl += gridDim.y)
  for (uint32_t base = tl * kEmitTile, tend = min(n, (tl + 1) * kEmitTile); base < tend; base += NT) {
    const uint32_t nb = min((uint32_t)NT, tend - base);
    uint32_t cnt = 0;
    if ((uint32_t)t < nb) {
      sh_c[t] = cmds[sg.cmd_off + base + t];
      sh_p[t] = cmd_pos[sg.cmd_off + base + t];
      cnt = item_count(sh_c[t]);
    }
    uint32_t off, nitems;
    Scan(scan_tmp).ExclusiveSum(cnt, off, nitems);
    map.off[t] = off;
    if (t == 0) map.off[nb] = nitems;
    __syncthreads();
    uint32_t bits = 0;
    for (uint32_t i = t; i < nitems; i += NT) {
      const uint32_t j = map.find(i, nb);
      const uint32_t p = sh_p[j];
      bits += item_bits(cd, mb, sh_cmap, lut, jb, sh_c[j], p, sg, sh_u, base + j, i - map.off[j]);
    }
    const uint32_t sum = Reduce(red_tmp).Sum(bits);
    if (t == 0) {
      tile += sum;
      total += sum;
      if (base + NT >= tend) {
        tb[tl] = tile;
        tile = 0;
      }
    }
    __syncthreads();
  }
  if (t == 0) atomicAdd(reinterpret_cast<unsigned long long *>(&sg.bits), total);
}

// ---------------------------------------------------------------- offsets: wave per stream
// Bit offsets of the metablocks and segments: prefix sums of the sizes, 64 segments a step.
__global__ __launch_bounds__(64) void offsets_kernel(Job *jobs, int njobs, Mb *mbs, Seg *segs, uint8_t *out) {
  const int j = blockIdx.x, lane = threadIdx.x;
  if (j >= njobs) return;
  Job &jb = jobs[j];
  if (jb.uncompressed) return;
  uint64_t pos = jb.parts ? jb.idx_bits : 0;   // window bits + part index block first
  for (uint32_t m = 0; m < jb.nmb; m++) {
    Mb &mb = mbs[jb.mb_base + m];
    if (lane == 0) mb.bit_off = pos;
    uint64_t hb = lane < kTreeSlots ? mb.tree_bits[lane] : 0;
    for (int q = lane + 64; q < kTreeSlots; q += 64) hb += mb.tree_bits[q];
    for (int o = 32; o; o >>= 1) hb += __shfl_xor(hb, o);
    pos += mb.hdr_bits + hb;
    const uint32_t end = mb.first_seg + mb.nseg;
    for (uint32_t c0 = mb.first_seg; c0 < end; c0 += 64) {
      const uint32_t s = c0 + lane;
      const uint64_t bits = s < end ? segs[s].bits : 0;
      uint64_t inc = bits;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint64_t y = __shfl_up(inc, o);
        if (lane >= o) inc += y;
      }
      if (s < end) segs[s].bit_off = pos + inc - bits;
      pos += __shfl(inc, 63);
    }
    if (mb.is_last) pos = (pos + 7) & ~7ull;
  }
  if (lane != 0) return;
  const uint64_t trailer = pos;
  if (!jb.final_) pos = (pos + 6 + 7) & ~7ull;   // empty metadata block: ISLAST 0, MNIBBLES 0, MSKIPBYTES 0
  // the stored form is never larger than n + 5 bytes per 16 MiB block + window header + tail
  const uint64_t stored_bits = 8ull * ((uint64_t)jb.n + 5ull * ((jb.n >> 24) + 1) + 4);
  if (pos > stored_bits || (pos >> 3) + 8 > jb.out_cap) {
    jb.uncompressed = 2;   // emit stored metablocks instead
    for (int q = 0; q < 4; q++) jb.dc_out[q] = jb.dc_in[q];
    return;
  }
  if (!jb.final_) {   // bits 0,1,1,0,0,0 = 6
    uint32_t *w = reinterpret_cast<uint32_t *>(out + jb.out_off);
    const uint64_t v = 6ull << (trailer & 31);
    atomicOr(w + (trailer >> 5), (uint32_t)v);
    if ((uint32_t)(v >> 32)) atomicOr(w + (trailer >> 5) + 1, (uint32_t)(v >> 32));
  }
  jb.total_bits = pos;
}

// ---------------------------------------------------------------- launchers
void launch_carry(hipStream_t st, Job *jobs, int njobs, Seg *segs, const Mb *mbs) {
  hipLaunchKernelGGL(carry_kernel, dim3(njobs), dim3(64), 0, st, jobs, njobs, segs, mbs);
}
void launch_codes(hipStream_t st, const Job *jobs, const Seg *segs, const Mb *mbs, int nsegs, const RawCmd *raw, Cmd *cmds,
                  uint32_t *cmd_pos, Unit *units, uint32_t *unit_h) {
  // 512 threads: the 35 KiB unit histograms allow four blocks (32 waves) per CU (MIB_CODES_NT overrides)
  static const int nt = knob("MIB_CODES_NT") ? atoi(knob("MIB_CODES_NT")) : 512;
  if (nt >= 512)
    hipLaunchKernelGGL(codes_kernel<512>, dim3(nsegs), dim3(512), 0, st, jobs, segs, mbs, raw, cmds, cmd_pos, units, unit_h);
  else
    hipLaunchKernelGGL(codes_kernel<256>, dim3(nsegs), dim3(256), 0, st, jobs, segs, mbs, raw, cmds, cmd_pos, units, unit_h);
}
void launch_split(hipStream_t st, hipStream_t side, const Job *jobs, Mb *mbs, int nmbs, Unit *units,
                  const uint32_t *unit_h, Codes *codes, int max_units, int max_short_units) {
  const SplitK sk = split_k();
  // a launch per state count: S = 4 for the blocks seeding at most four types, S = kMaxBT for
  // the rest (if any: literals of the metablocks of up to kSplitWideUnits units)
  const bool wide_short = std::max(sk.k[0], std::max(sk.k[1], sk.k[2])) > 4;
  const bool wide_long = std::max(std::min(sk.k[0], 4), std::max(sk.k[1], sk.k[2])) > 4;
  // (FONT metablocks cap literal types at 4 whatever k[0] is: with k[0] > 4 the S = 4 launch must
  // run for them even when no other block needs it -- ADVICE r4, an experiment-override case)
  const bool narrow = std::min(sk.k[0], std::min(sk.k[1], sk.k[2])) <= 4 || max_units > kSplitWideUnits || sk.k[0] > 4;
  const size_t lds4 = (size_t)std::max(1, std::min(max_units, kMaxUnits)) * 4 * sizeof(float);
  const size_t lds8 = (size_t)std::max(1, std::min(wide_long ? max_units : max_short_units, kMaxUnits)) * kMaxBT * sizeof(float);
  static const bool attr = [] {   // (dynamic LDS past 64 KiB: 16 MiB metablocks)
    hipFuncSetAttribute((const void *)split_kernel<1024, 4>, hipFuncAttributeMaxDynamicSharedMemorySize, kMaxUnits * 4 * 4);
    hipFuncSetAttribute((const void *)split_kernel<256, 4>, hipFuncAttributeMaxDynamicSharedMemorySize, kMaxUnits * 4 * 4);
    hipFuncSetAttribute((const void *)split_kernel<1024, kMaxBT>, hipFuncAttributeMaxDynamicSharedMemorySize, kMaxUnits * kMaxBT * 4);
    hipFuncSetAttribute((const void *)split_kernel<256, kMaxBT>, hipFuncAttributeMaxDynamicSharedMemorySize, kMaxUnits * kMaxBT * 4);
    return true;
  }();
  (void)attr;
  const bool few = nmbs * 3 <= 256;
  // (the two launches take disjoint (metablock, category) blocks: the four-type one runs on side)
  if (narrow) {
    if (few) hipLaunchKernelGGL((split_kernel<1024, 4>), dim3(nmbs * 3), dim3(1024), lds4, side, jobs, mbs, nmbs, units, unit_h, codes, sk);
    else hipLaunchKernelGGL((split_kernel<256, 4>), dim3(nmbs * 3), dim3(256), lds4, side, jobs, mbs, nmbs, units, unit_h, codes, sk);
  }
  if (wide_short || wide_long) {
    if (few) hipLaunchKernelGGL((split_kernel<1024, kMaxBT>), dim3(nmbs * 3), dim3(1024), lds8, st, jobs, mbs, nmbs, units, unit_h, codes, sk);
    else hipLaunchKernelGGL((split_kernel<256, kMaxBT>), dim3(nmbs * 3), dim3(256), lds8, st, jobs, mbs, nmbs, units, unit_h, codes, sk);
  }
  // the widening pass: after the four-type split of the command and distance
  // categories (on side), those whose split saved the most are split again with eight seeds,
  // and keep more than four types where that pays (the merge pass in split_kernel)
  static const bool widen = !knob("MIB_SPLIT_WIDEN") || atoi(knob("MIB_SPLIT_WIDEN")) != 0;   // (experiments: 0 off)
  if (widen && narrow && std::max(sk.k[1], sk.k[2]) <= 4) {
    SplitK wk = sk;
    wk.widen = 1;
    const size_t ldsw = (size_t)std::max(1, std::min(max_units, kMaxUnits)) * kMaxBT * sizeof(float);
    if (few) hipLaunchKernelGGL((split_kernel<1024, kMaxBT>), dim3(nmbs * 3), dim3(1024), ldsw, side, jobs, mbs, nmbs, units, unit_h, codes, wk);
    else hipLaunchKernelGGL((split_kernel<256, kMaxBT>), dim3(nmbs * 3), dim3(256), ldsw, side, jobs, mbs, nmbs, units, unit_h, codes, wk);
  }
}
void launch_histo(hipStream_t st, const Job *jobs, const Seg *segs, const Mb *mbs, int nsegs, const Cmd *cmds,
                  const uint32_t *cmd_pos, const Unit *units, uint32_t *hl, uint32_t *hc, uint32_t *hd) {
  // 1024 threads: the 64 KiB literal histogram allows two blocks per CU, so wider blocks are
  // what hides the per-literal gathers (C3 type_histo 9.6 -> 5.3 ms; MIB_HISTO_NT overrides)
  static const int nt = knob("MIB_HISTO_NT") ? atoi(knob("MIB_HISTO_NT")) : 1024;
  if (nt >= 1024)
    hipLaunchKernelGGL(histo_kernel<1024>, dim3(nsegs), dim3(1024), 0, st, jobs, segs, mbs, cmds, cmd_pos, units, hl, hc, hd);
  else if (nt >= 512)
    hipLaunchKernelGGL(histo_kernel<512>, dim3(nsegs), dim3(512), 0, st, jobs, segs, mbs, cmds, cmd_pos, units, hl, hc, hd);
  else
    hipLaunchKernelGGL(histo_kernel<256>, dim3(nsegs), dim3(256), 0, st, jobs, segs, mbs, cmds, cmd_pos, units, hl, hc, hd);
}
void launch_dist_ring(hipStream_t st, Job *jobs, int njobs, const Seg *segs, const Cmd *cmds) {
  hipLaunchKernelGGL(dist_ring_kernel, dim3((njobs + 63) / 64), dim3(64), 0, st, jobs, njobs, segs, cmds);
}
void launch_context_mode(hipStream_t st, const Job *jobs, Mb *mbs, int nmbs) {
  static const int force = knob("MIB_CTX_MODE") ? atoi(knob("MIB_CTX_MODE")) & 3 : -1;   // experiments
  hipLaunchKernelGGL(context_mode_kernel, dim3(nmbs), dim3(64), 0, st, jobs, mbs, nmbs, force);
}
// Literal prefix codes per metablock: at most kLitTreeCap.  The decoder keeps a metablock's
// tables in its LDS table area only when they fit (12,224 entries, >= 256 per code); past
// that every symbol lookup is an HBM load.  With up to 64 codes some C3 fonts overflowed it,
// and the batch kernel waits for its slowest stream: C3 decode 76 -> 46 ms at 32 codes, and
// the stream is smaller too (0.4585 -> 0.4582: fewer codes to send); 24: 0.45816 / 45.6 ms;
// C4 never needs more than 24.  MIB_LIT_TREES overrides (1..64; 1: one code per block type,
// context-free literals).
constexpr int kLitTreeCap = 24;
int lit_tree_cap() {
  static const int cap = knob("MIB_LIT_TREES") ? std::min(kMaxLitTrees, std::max(1, atoi(knob("MIB_LIT_TREES")))) : kLitTreeCap;
  return cap;
}
void launch_cluster(hipStream_t st, const Job *jobs, Mb *mbs, int nmbs, uint32_t *hl, uint32_t *hd) {
  const SplitK sk = split_k();
  static const int kd = knob("MIB_TYPE_SIZING") ? sk.k[2] : kMaxBT;   // (the widening pass may leave more than sk.k[2] distance types)
  hipLaunchKernelGGL(cluster_kernel, dim3(nmbs * (sk.k[0] + 4)), dim3(kCluT), 0, st, jobs, mbs, nmbs, hl, hd, lit_tree_cap(),
                     sk.k[0], kd);
}
void launch_huffman(hipStream_t st, hipStream_t side, const Job *jobs, Mb *mbs, int nmbs, const uint32_t *hl,
                    const uint32_t *hc, const uint32_t *hd, Codes *codes, uint8_t *trees, uint8_t *hdr) {
  // one launch for every slot (two launches by alphabet size, the literal one with half the LDS,
  // were measured: C4 6.0 -> 5.5 ms but C3 8.9 -> 10.2 -- the command / distance blocks, the
  // longest, then ran as a tail of their own)
  // blocks per metablock: the literal codes (at most the cap, or one per literal type), one per
  // command type, the distance (type, cluster) slots
  const SplitK sk = split_k();
  // (command / distance: kMaxBT types, the widening pass may leave more than sk.k[1], sk.k[2])
  static const int kc = knob("MIB_TYPE_SIZING") ? sk.k[1] : kMaxBT, kdt = knob("MIB_TYPE_SIZING") ? sk.k[2] : kMaxBT;   // (experiments)
  (void)kdt;
  const int nl = std::max(lit_tree_cap(), sk.k[0]), nr = nl + 4 + 4 * kDistCtx;   // (types 4..kc-1: second items)
  hipLaunchKernelGGL(huffman_kernel<704>, dim3(nmbs * nr), dim3(64), 0, st, jobs, mbs, nmbs, hl, hc, hd, codes, trees, nl, kc, nr);
  // the header reads the split's and the clustering's results, not the prefix codes (it writes
  // Mb.hdr_bits and the block-split codes, huffman_kernel Mb.tree_bits and the other codes)
  hipLaunchKernelGGL(mb_header_kernel, dim3(nmbs), dim3(64), 0, side, jobs, mbs, nmbs, hdr, codes);
}
void launch_sizes(hipStream_t st, const Job *jobs, Seg *segs, const Mb *mbs, int nsegs, const Cmd *cmds,
                  const uint32_t *cmd_pos, const Codes *codes, const Unit *units, uint32_t *tile_bits) {
  static const int nt = knob("MIB_SIZES_NT") ? atoi(knob("MIB_SIZES_NT")) : 512;   // (MIB_SIZES_NT overrides)
  // blocks per segment: enough for ~2,048 blocks, as launch_emit
  static const int target = knob("MIB_EMIT_BLOCKS") ? std::max(1, atoi(knob("MIB_EMIT_BLOCKS"))) : 2048;
  const dim3 grid(nsegs, std::min(kEmitTiles, std::max(1, (target + nsegs - 1) / std::max(nsegs, 1))));
  if (nt >= 512)
    hipLaunchKernelGGL(sizes_kernel<512>, grid, dim3(512), 0, st, jobs, segs, mbs, cmds, cmd_pos, codes, units, tile_bits);
  else
    hipLaunchKernelGGL(sizes_kernel<256>, grid, dim3(256), 0, st, jobs, segs, mbs, cmds, cmd_pos, codes, units, tile_bits);
}
void launch_offsets(hipStream_t st, Job *jobs, int njobs, Mb *mbs, Seg *segs, uint8_t *out) {
  hipLaunchKernelGGL(offsets_kernel, dim3(njobs), dim3(64), 0, st, jobs, njobs, mbs, segs, out);
}

}  // namespace enc
}  // namespace mib
#ifdef MIB_PROF
extern "C" int mib_debug_read_huff_prof(unsigned long long *out) {
  hipMemcpyFromSymbol(out, HIP_SYMBOL(mib::enc::g_huff_prof), sizeof(unsigned long long) * 12);
  unsigned long long z[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  hipMemcpyToSymbol(HIP_SYMBOL(mib::enc::g_huff_prof), z, sizeof(z));
  return 0;
}
#endif
#ifdef MIB_PROF
extern "C" int mib_debug_read_split_prof(unsigned long long *out) {
  hipMemcpyFromSymbol(out, HIP_SYMBOL(mib::enc::g_split_prof), sizeof(unsigned long long) * 8);
  unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  hipMemcpyToSymbol(HIP_SYMBOL(mib::enc::g_split_prof), z, sizeof(z));
  return 0;
}
#endif
#ifdef MIB_PROF
extern "C" int mib_debug_read_clu_prof(unsigned long long *out) {
  hipMemcpyFromSymbol(out, HIP_SYMBOL(mib::enc::g_clu_prof), sizeof(unsigned long long) * 8);
  unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  hipMemcpyToSymbol(HIP_SYMBOL(mib::enc::g_clu_prof), z, sizeof(z));
  return 0;
}
#endif
