// The parse: the wave-per-segment shortest-path DP and the
// backtrack that turns its choices into commands.
#include <hipcub/hipcub.hpp>
#include <cstdlib>

#include "enc_common.h"

namespace mib {
namespace enc {

// ---------------------------------------------------------------- 3. DP parse
// Shortest path over positions (updateNodes / computeShortestPathFromNodes,
// backward-references-hq.ts:267-406): node i holds the cheapest cost of reaching i, the
// insert length since the last copy, and the path's last distance.  Edges out of i: one
// literal, and the staircase matches of i (the shortest distance covering each length),
// priced with short code 0 when the distance is the path's last distance.  A copy longer
// than kLongCopy is taken outright and the parse jumps to its end, as the reference does
// (:518-533).
//
// kS segments per wave, kL = 64 / kS lanes each, the pending nodes in REGISTERS: a segment
// is parsed in batches of kL positions starting at i0, and lane j of the segment's lane
// group in chunk k holds node i0 + kL k + j.  Relaxing the edge of length l out of
// i = i0 + off lands in chunk (off + l) / kL, lane (off + l) % kL: every lane relaxes the one
// length that maps to it -- a lane-local compare/select, no LDS round trip -- and only the
// chunks holding lengths 0..maxlen are touched.  The segments of a wave advance in lockstep
// (one position each per step), so one VALU instruction relaxes kS positions: text's
// staircases are short (maxlen ~ 10-30), and a 64-lane chunk per position left most lanes
// idle.  Everything per segment is lane-group-uniform and lives in VGPRs; control flow that
// differs between the segments (a segment's end, a long copy, a batch end) is predicated.
// Node i is fetched with ds_bpermute from its lane; at a batch end the segment's chunks move
// down by one (chunk 0 is all consumed nodes).
//
// The length-dependent half of a copy's price (its copy code's extra bits, the command code
// it forms with the insert code, with and without short code 0) comes from a per-segment LDS
// table indexed by (insert code, copy code), fp16 pairs, and a length -> copy code table.
// Per-position inputs (matches, distance-cost codes, literal cost) are staged one lane per
// position into LDS, loaded a batch ahead, and read back with one broadcast read per
// segment; the batch's choices are collected per lane and stored as one coalesced write.
#ifdef MIB_PROF   // timing experiment: cycles in staging / node read / long copies / relaxation; counts
__device__ unsigned long long g_dp_prof[8];
#define DPMARK(slot)                                  \
  do {                                                \
    const uint64_t t_ = __builtin_amdgcn_s_memtime(); \
    prof[slot] += t_ - pt0;                           \
    pt0 = t_;                                         \
  } while (0)
#define DPCOUNT(slot, v) prof[slot] += (v)
#else
#define DPMARK(slot) do {} while (0)
#define DPCOUNT(slot, v) do {} while (0)
#endif
// kS is a template parameter: 2 segments per wave (32 lanes each) for batches with enough
// segments to fill the chip, 1 (64 lanes) when there are fewer waves than SIMDs (one long
// stream): a step then relaxes twice the lengths per instruction on a wave that would
// otherwise share its SIMD with nothing.
constexpr int kDpWaves = 4;           // waves per workgroup, sharing the length table
constexpr int kLenTab = kLongCopy + 1;
constexpr int kInsTab = 256;            // insert lengths with a table entry
constexpr float kInf = 3.0e38f;
constexpr uint32_t kCostLast = 255;   // cost code of a match at the path's last distance
// LDS per workgroup sized for five workgroups per CU (the price table keeps kPtabW of its 24
// columns: copy codes of relaxed lengths <= kLongCopy stay below it; literal costs as 16-bit
// fixed point, which they are), VGPRs for MIB_DP_OCC waves per SIMD: the step is a dependent
// chain (node fetch by ds_bpermute, two table reads, the relaxation's compares), so more waves
// hide more of it -- five alone (C4 dp 106.5 -> 100.7 ms), but four beside the other encode
// lanes' kernels (r04o: C4 2,937 vs 2,861 MB/s).
#ifndef MIB_DP_OCC
#define MIB_DP_OCC 4   // (A/B builds: 5; with two encode lanes 4 is faster, r04o)
#endif
constexpr int kDpWavesPerSimd = MIB_DP_OCC;
#ifndef MIB_DP_OCC_KS4
#define MIB_DP_OCC_KS4 MIB_DP_OCC   // (A/B builds: the four-segment build's occupancy target)
#endif
constexpr int kPtabW = 20;
constexpr int kRepLen = 16;   // last-distance copies relaxed up to this length (<= the lanes per segment)
static_assert(kLongCopy <= 325, "copy codes of lengths <= 325 are < 20 (command.ts getCopyLengthCode)");

typedef const __attribute__((address_space(1))) uint8_t GCU8;

// kCopyExtra / kInsExtra in closed form (no table loads on the serial path)
__device__ __forceinline__ uint32_t copy_extra(int cc) { return cc < 8 ? 0u : cc < 18 ? (uint32_t)(cc - 6) >> 1 : cc < 23 ? (uint32_t)(cc - 12) : 24u; }
__device__ __forceinline__ uint32_t ins_extra(int ic) {
  return ic < 6 ? 0u : ic < 16 ? (uint32_t)(ic - 4) >> 1 : ic < 21 ? (uint32_t)(ic - 10) : ic == 21 ? 12u : ic == 22 ? 14u : 24u;
}
// iteration-0 cost model (zopfli-cost-model.ts: costCmd = log2(11 + code), costDist = log2(20 + code))
__device__ __forceinline__ float cmd_cost(int cmd) { return __builtin_amdgcn_logf(11.f + (float)cmd); }
__device__ __forceinline__ float dist_sym_cost(uint32_t code) { return __builtin_amdgcn_logf(20.f + (float)min(code, 127u)); }
// the second iteration's prices come from the workgroup's CostModel (null: iteration 0)
__device__ __forceinline__ float cmd_price(int cmd, const CostModel *cm) { return cm ? cm->cmd[cmd] : cmd_cost(cmd); }
__device__ __forceinline__ float dist_price(uint32_t code, const CostModel *cm) {
  return cm ? cm->dist[min(code, 127u)] : dist_sym_cost(code);
}
// the length-dependent price of a copy with copy code cc after insert code ic: with an
// explicit distance (its symbol cost added by the caller), and with short code 0 (complete)
__device__ __forceinline__ float copy_price(int ic, int cc, bool last, float dist0, const CostModel *cm) {
  const int cmd = combine_codes(ic, cc, last);
  return (float)copy_extra(cc) + cmd_price(cmd, cm) + (last && cmd >= 128 ? dist0 : 0.f);
}

// ins_code / ins_extra (command.ts:29-64) without branches: the node's insert length is
// lane-group-uniform but not wave-uniform here, so a branchy form would run every arm
__device__ __forceinline__ int ins_code_sel(uint32_t n) {
  const uint32_t a = n - 2u, lga = 31u - (uint32_t)__clz((int)(a | 1u));          // n in [6, 130)
  const uint32_t nb = lga - 1u;
  const uint32_t mid = (nb << 1) + (a >> nb) + 2u;
  const uint32_t hi = 31u - (uint32_t)__clz((int)((n - 66u) | 1u)) + 10u;          // n in [130, 2114)
  uint32_t c = n < 6u ? n : n < 130u ? mid : n < 2114u ? hi : n < 6210u ? 21u : n < 22594u ? 22u : 23u;
  return (int)c;
}
__device__ __forceinline__ uint32_t ins_extra_sel(int ic) {
  const uint32_t u = (uint32_t)ic;
  return u < 6u ? 0u : u < 16u ? (u - 4u) >> 1 : u < 21u ? u - 10u : u == 21u ? 12u : u == 22u ? 14u : 24u;
}

struct Staged {   // one position's parse inputs as loaded
  uint32_t m[kMaxMatches];
  uint32_t nm;
  uint32_t lit;
  uint32_t w0, w1;   // (KC) the position's first 8 bytes: words[g], words[g + 4]
};
template <bool KC>
__device__ __forceinline__ void load_staged(Staged &st, const uint32_t *matches, const uint8_t *data, const uint32_t *words,
                                            uint32_t g, uint32_t p) {
  st.lit = data[p];
  rec_load(matches + (uint64_t)g * kMatchRec, st.m);   // 0 = no entry
  st.nm = 0;
#pragma unroll
  for (int q = 0; q < kMaxMatches; q++) st.nm += st.m[q] != 0u;
  if (KC) {
    st.w0 = words[g];
    st.w1 = words[g + 4];
  }
}
struct alignas(16) StageEnt {   // one position's parse inputs in LDS (48 B: two b128 reads and a b64)
  uint32_t m[kMaxMatches];   // (clipped length << 24) | distance, 0 = none
  uint32_t mc[kMaxMatches];  // distance | distance-cost code << 24 (quarter bits)
  uint32_t info;             // nm | maxlen << 8 | shortest usable length << 16
  float lc;                  // literal cost
  uint32_t w[2];             // (KC) the position's first 8 bytes, for its distance-cache candidates
};
__device__ __forceinline__ uint64_t choice_of(uint32_t d, uint32_t m) {   // (distance << 32) | length, 0 = literal
  const uint32_t cl = (m >> 16) ? 0u : m & 0xFFFF;   // (a literal edge: insert length << 16 | its codes)
  return cl ? (((uint64_t)d << 32) | cl) : 0ull;
}
__device__ __forceinline__ uint32_t bperm(uint32_t lane_src, uint32_t v) {
  return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(lane_src << 2), (int)v);
}
// quad permutes (DPP, no LDS): the distance ring lives in the lanes of each quad, entry q in
// lane q of the quad
__device__ __forceinline__ uint32_t quad_entry0(uint32_t v) { return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x00, 0xF, 0xF, false); }
__device__ __forceinline__ uint32_t quad_entry1(uint32_t v) { return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x55, 0xF, 0xF, false); }
__device__ __forceinline__ uint32_t quad_shift1(uint32_t v) { return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x90, 0xF, 0xF, false); }

// ---------------------------------------------------------------- distance-cache candidates
// (KC; SURVEY a6, backward-references-hq.ts:309-345, computeDistanceCache :213-234).  Every
// node's path has a decoder distance ring (the last four distances its copies pushed, RFC 7932
// section 4); short code j (1..15) names ring entry kIdx[j] plus kOff[j].  The pending nodes
// cannot carry four distances each in registers, so the ring is kept per POSITION of the path
// already decided: when node x is final (it has become the current node), its ring follows
// from its edge -- a literal keeps node x-1's ring, a copy pushes its distance on its
// predecessor's ring (unless it repeats entry 0; a dictionary word pushes nothing) -- and is
// stored in a 256-position history per lane group (global memory, L1/L2 resident); a copy
// node's predecessor is at most kLongCopy back.  Pipelined so that no step waits on memory:
//   step of node i:  fetch node i, load its predecessor's ring from the history (copy edge);
//                    ring of node i-1 from the load issued one step ago, stored;
//                    node i-1's 15 candidate distances (a lane each), their source words
//                    loaded (words[]: each position's 4 bytes, one aligned load per word);
//                    node i-2's candidates (loaded one step ago) measured over 8 bytes and
//                    relaxed out of node i-2 for lengths 4..R (the reference's minimum: >= 4),
//                    priced with the short code's distance symbol.
// Code 0 (entry 0, no offset) is KR's last-distance copy when that is built, else lane 0 here.
// The ring at a segment / piece start is unknown: entries 0 offer nothing until the path's
// own copies fill them.  codes_kernel assigns the real short codes afterwards from the decoder's
// exact ring (ring_scan_kernel), so a candidate the parse priced is coded as priced except near
// a piece start.
constexpr uint32_t kHistPos = 256;      // ring history per lane group (> kLongCopy)
static_assert(kHistPos > (uint32_t)kLongCopy, "a copy's predecessor must still be in the ring history");

// KM: the second iteration (prices from the stream's CostModel; a separate build, so
// profiles tell the two passes apart).  KD: some stream has a custom dictionary (records with
// kCDictMark; a separate build, so the common case pays nothing for it).  KR: the parse relaxes
// last-distance copies (rp_d below; FONT mode: C3 -1 % bytes, text -0.1 %, a separate build so
// text pays nothing for it)
template <int KS, bool KM, bool KD, bool KR, bool KC>
__global__ __launch_bounds__(64 * kDpWaves, KS == 4 ? MIB_DP_OCC_KS4 : (KC && KS == 2) ? 3 : kDpWavesPerSimd) void dp_kernel(const Job *jobs, const Seg *segs, int nsegs,
                                                           const uint32_t *lit_histo, const CostModel *model,
                                                           const uint32_t *matches,
                                                           uint64_t *choice /* per position+1 */, float cmd_pen, int use_rep,
                                                           const uint32_t *pwords, uint32_t *ring_hist, const Mb *mbs,
                                                           int kc_split) {
  constexpr int kS = KS;                // segments per wave
  constexpr int kL = 64 / kS;           // lanes per segment
  constexpr int kC = (kL - 1 + kLongCopy) / kL + 1;   // chunks: batch offset (< kL) + longest relaxed length
  static_assert(kL - 1 + kLongCopy < kL * kC, "every relaxed length must land in a chunk");
  static_assert(kRepLen <= kL, "a last-distance copy is measured by one lane per byte");
  static_assert(!KC || kL >= 16, "a lane per distance-cache candidate");
  constexpr uint64_t kLaneMask = kL == 64 ? ~0ull : ((1ull << kL) - 1);
  __shared__ uint32_t ptab_all[kDpWaves * kS][24 * kPtabW];   // per segment: (insert code, copy code) -> fp16 (explicit distance) | fp16 (short code 0) << 16
  __shared__ uint8_t cctab[kLenTab];                       // length -> copy code
  __shared__ uint16_t itab[kInsTab];                       // insert length -> insert code | its extra bits << 8
  __shared__ uint16_t litc_all[kDpWaves * kS][256];   // literal costs in 1/256 bits (exact: they are quantised so)
  // (one spare entry per 32 lanes, per 16 with four segments: the entries the segments read at
  // the same offset in one instruction -- i and 32 + i, or i, 16 + i, 32 + i, 48 + i -- fall 12
  // banks apart instead of on the same banks: 16 entries are 192 words, a multiple of the 64)
  constexpr int kPadSh = KS == 4 ? 4 : 5;
  __shared__ StageEnt stg_all[kDpWaves][64 + (64 >> kPadSh)];
  for (int t = threadIdx.x; t < kLenTab; t += 64 * kDpWaves) cctab[t] = (uint8_t)(t >= 2 ? copy_code((uint32_t)t) : 0);
  for (int t = threadIdx.x; t < kInsTab; t += 64 * kDpWaves) {
    const int ic = ins_code((uint32_t)t);
    itab[t] = (uint16_t)(ic | (ins_extra(ic) << 8));
  }
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63, w = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const uint32_t h = lane / kL, hl = lane % kL, hbase = h * kL;
  const int sgi = (blockIdx.x * kDpWaves + (int)w) * kS + (int)h;
  StageEnt *stg = stg_all[w];
  uint16_t *litc = litc_all[w * kS + h];
  uint32_t *ptab = ptab_all[w * kS + h];
  // this lane group's segment (a = b: nothing to parse)
  uint32_t a = 0, b = 0, gbase = 0, job = 0;
  const uint8_t *data = nullptr;
  int ndirect = 0, npostfix = 0;
  uint32_t parts = 0, abs0 = 0, wabs = 0, pbits = 16, plag = 0, maxback = 0, cdl = 0;
  bool words = false;
  if (sgi < nsegs) {
    const Seg &sg = segs[sgi];
    const Job &jb = jobs[sg.job];
    a = sg.start;
    b = sg.end;
    gbase = jb.pos_base;
    job = sg.job;
    data = jb.data;
    ndirect = (int)jb.ndirect;
    npostfix = (int)jb.npostfix;
    parts = jb.parts;
    abs0 = jb.abs_base;   // (part alignment: mod 2^32 is exact)
    wabs = jb.win_abs;     // (dictionary distances: saturated, no wrap past 4 GiB)
    pbits = jb.part_bits;
    plag = jb.part_lag;
    maxback = (1u << jb.lgwin) - 16;
    words = jb.dict != 0;
    cdl = jb.cdict ? jb.cdict_len : 0u;
  }
  // kc_split: the candidates' build takes the segments whose metablock's literals are not UTF-8
  // text (context_mode_kernel), the other build the rest (text: the candidates changed C4 by
  // +0.01 % bytes, r06b)
  if (kc_split && a < b && (mbs[segs[sgi].mb].ctx_mode == 2u) == KC) a = b;
  if (__ballot(a < b) == 0) return;
  // prices: iteration 0 from zopfli-cost-model.ts's initial model, iteration 1 from the
  // stream's CostModel (per segment tables: a wave's segments may be different streams)
  const CostModel *cm = (KM && a < b) ? model + job : nullptr;
  const float dist0 = dist_price(0, cm);
  if (a < b)
    for (uint32_t t = hl; t < 24 * kPtabW; t += kL) {
      const int ic = (int)(t / kPtabW), cc = (int)(t % kPtabW);
      const _Float16 x = (_Float16)(copy_price(ic, cc, false, dist0, cm) + cmd_pen),
                     y = (_Float16)(copy_price(ic, cc, true, dist0, cm) + cmd_pen);
      ptab[t] = (uint32_t)__builtin_bit_cast(uint16_t, x) | ((uint32_t)__builtin_bit_cast(uint16_t, y) << 16);
    }
  // literal costs: iteration 0 from the stream's order-0 histogram (zopfli-cost-model.ts:
  // 163-189), iteration 1 from the model
  if (cm) {
    if (a < b)
      for (uint32_t k = hl; k < 256; k += kL)
        litc[k] = (uint16_t)(uint32_t)(fminf(fmaxf(cm->lit[k], 1.f), 255.f) * 256.f);
  } else {
    uint32_t part = 0;
    if (a < b)
      for (uint32_t k = hl; k < 256; k += kL) part += lit_histo[job * 256 + k];
    for (int o = kL / 2; o; o >>= 1) part += __shfl_xor(part, o);
    const float lt = log2f((float)max(part, 1u));
    if (a < b)
      for (uint32_t k = hl; k < 256; k += kL) {
        const uint32_t c = lit_histo[job * 256 + k];
        const float v = c ? lt - log2f((float)c) : lt + 2.f;
        litc[k] = (uint16_t)(uint32_t)(fminf(fmaxf(v, 1.f), 255.f) * 256.f);
      }
  }
  wave_sync();
  // the pending nodes: cost, last distance, and the copy length that reached it, or (a literal
  // edge) insert length << 16 | its insert code | the code's extra bits << 8
  float wc[kC];
  uint32_t wd[kC], wm[kC];
#pragma unroll
  for (int c = 0; c < kC; c++) {
    wc[c] = kInf;
    wd[c] = wm[c] = 0;
  }
  if (hl == 0) wc[0] = 0.f;   // node a
  Staged pf;
  uint32_t pf_at = a;
  if (a + hl < b) load_staged<KC>(pf, matches, data, pwords, gbase + a + hl, a + hl);
  uint32_t chd = 0, chm = 0;   // choices of the batch
  // the pending last-distance candidate (a6): node j reached by a literal, with last distance
  // rp_d, loads the bytes at j + hl and j - rp_d + hl in its step; the step of node j + 1 (the
  // loads' latency hidden behind one step) measures the match and relaxes lengths 2 .. R out
  // of j, priced with short code 0 (rp_base / rp_ic: node j's cost + insert extra, insert code)
  uint32_t rp_d = 0, rp_ic = 0, rp_cb = 0, rp_sb = 1;
  float rp_base = 0.f;
  // distance-cache candidates (KC, see above): this lane's short code (lanes 0..15 of the group);
  // the ring entry q = lane % 4 of each quad.  State packed to keep the build's registers down.
  const uint32_t cj = hl & 15u, rq = hl & 3u;
  const bool clane = KC && hl < 16u && (!KR || cj != 0u);
  const float ccost = KC ? dist_price(cj, cm) : 0.f;   // its distance symbol (short codes carry no extra bits)
  const uint32_t hoff = (uint32_t)sgi * (kHistPos * 4);   // this lane group's ring history: 256 positions x 4 distances
  // kf: bits 0-1 node i-1's edge (0 none, 1 literal, 2 copy); bit 2 the next node ends a long
  // copy (its ring is rg); bit 3 node i-2's candidates are in flight; bits 8-15 node i-1's insert
  // code, bits 16-23 node i-2's
  uint32_t kf = 0;
  uint32_t kp_ld = 0, kp_h = 0;   // node i-1's distance, its predecessor's ring entry rq (copy edge)
  float kp_base = 0.f;            // node i-1's cost + insert extra
  uint32_t rg = 0;                // ring entry rq of node i-2 (after the ring step: of node i-1)
  // node i-2's candidates: distance (0: none), source words, own words, length cap, its match
  // record (the staircase: a match's full length at the candidate's distance)
  uint32_t cq_d = 0, cq_w0 = 0, cq_w1 = 0, cq_c0 = 0, cq_c1 = 0, cq_lim = 0;
  uint32_t cq_m[kMaxMatches] = {};
  const int coff = cj < 4u ? 0 : (int)(((cj - 4u) % 6u) / 2u + 1u) * (((cj - 4u) & 1u) ? 1 : -1);   // short code cj's offset
  float cq_base = 0.f;
  auto words_on_ring = [&](uint32_t dd) { return words && is_dict(dd); };
  auto ring_step = [&](uint32_t kind, uint32_t dd, uint32_t h, uint32_t prev) -> uint32_t {
    const uint32_t v = kind == 2u ? h : prev;
    const uint32_t v0 = quad_entry0(v), vm = quad_shift1(v);
    const bool word = words_on_ring(dd);
    const bool push = kind == 2u && dd != v0 && !word;
    return push ? (rq == 0u ? dd : vm) : (kind == 2u && word && rq == 0u) ? dd : v;
  };
  uint32_t i = a, i0 = a;
  bool done = a >= b;
#ifdef MIB_PROF
  uint64_t prof[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  uint64_t pt0 = __builtin_amdgcn_s_memtime();
#endif
  // stage the batch starting at i0 (the window's chunk 0 starts there) into this lane's entry
  auto stage = [&]() {
    Staged cur;
    cur.nm = 0;
    cur.lit = 0;
    cur.w0 = cur.w1 = 0;
    if (pf_at == i0) {
      cur = pf;
    } else if (i0 + hl < b) {   // the parse jumped past the prefetched batch
      load_staged<KC>(cur, matches, data, pwords, gbase + i0 + hl, i0 + hl);
    }
    const uint32_t nx = i0 + kL;
    if (nx + hl < b) load_staged<KC>(pf, matches, data, pwords, gbase + nx + hl, nx + hl);
    pf_at = nx;
    const uint32_t p = i0 + hl;
    const uint32_t nm = p < b ? cur.nm : 0u;
    StageEnt e;
    e.lc = p < b ? (float)litc[cur.lit] * (1.f / 256.f) : 0.f;
    uint32_t maxlen = 0, word = 0;
#pragma unroll
    for (int q = 0; q < kMaxMatches; q++) {
      e.m[q] = 0;
      e.mc[q] = 0;
      if ((uint32_t)q < nm) {
        uint32_t extra;
        uint32_t md = match_dist(cur.m[q]), d = md;
        uint32_t ln = min(match_length(cur.m[q]), b - p);
        if (KD && md == kCDictMark) {   // a custom-dictionary copy (the only entry): its exact length
          word = ln == match_length(cur.m[q]) ? 1u : 0u;   // cut by the segment end: unusable
          ln = word ? ln : 0u;
          d = min(wabs + p, maxback) + ln;
        } else if (words && is_dict(md)) {   // a dictionary word (the only entry): its distance at p, its exact length
          d = min(wabs + p, maxback) + 1 + cdl + (md & 0x7FF);   // (a custom dictionary comes first, engine.ts:907)
          md = d | kDictFlag;
          word = ln == match_length(cur.m[q]) ? 1u : 0u;   // cut by the segment end: unusable
          ln = word ? ln : 0u;
        }
        const uint32_t dp = dist_prefix(d + 15, ndirect, npostfix, &extra);
        e.m[q] = (ln << 24) | md;
        const float dc = (float)(dp >> 10) + dist_price(dp & 0x3FFu, cm);
        e.mc[q] = md | (min((uint32_t)(dc * 4.f + 0.5f), kCostLast - 1) << 24);
        maxlen = ln;
      }
    }
    e.info = (maxlen ? nm : 0u) | (maxlen << 8) | ((word ? maxlen : 2u) << 16);   // | the shortest usable length
    e.w[0] = KC ? cur.w0 : 0u;
    e.w[1] = KC ? cur.w1 : 0u;
    stg[lane + (lane >> kPadSh)] = e;
  };
  if (!done) stage();
  wave_sync();
  DPMARK(0);
  for (;;) {
    if (__ballot(!done) == 0) break;
    const uint32_t off = i - i0;   // < kL
    // ---- node i of each segment, from its lane of chunk 0
    const uint32_t src = hbase + (off & (kL - 1));
    const float ci = __uint_as_float(bperm(src, __float_as_uint(wc[0])));
    const uint32_t ld = bperm(src, wd[0]), mm = bperm(src, wm[0]);
    if (!done) {
      chd = hl == off ? ld : chd;
      chm = hl == off ? mm : chm;
      if (i == b) {   // the last batch, through node b
        const uint32_t p = i0 + hl;
        if (p <= b && p != a) choice[gbase + p] = choice_of(chd, chm);
        done = true;
      }
    }
    const bool act = !done;
    const StageEnt &e = stg[src + (src >> kPadSh)];
    const uint32_t info = e.info;
    const uint32_t nm = act ? (info & 0xFF) : 0u, maxlen = act ? ((info >> 8) & 0xFF) : 0u;
    const uint32_t minlen = info >> 16;   // 2, or a dictionary word's length: that length only
    const float litcost = e.lc;
    const uint32_t ins = mm >> 16;
    // the node's insert code and extra bits came with it (its literal edge carried them: see
    // nx); a copy's end node has none
    const int ic = ins ? (int)(mm & 0xFF) : 0;
    const uint32_t iextra = ins ? (mm >> 8) & 0xFF : 0u;
    // the codes of insert length ins + 1, for the literal edge out of i: looked up now, beside
    // the copy prices' lookup, so the next step has no insert-code lookup on its serial path
    const uint32_t ins1 = min(ins + 1, 65535u);
    uint32_t nx;
    if (__builtin_expect(ins1 < (uint32_t)kInsTab, 1)) {
      nx = itab[ins1];
    } else {
      const int c1 = ins_code_sel(ins1);
      nx = (uint32_t)c1 | (ins_extra_sel(c1) << 8);
    }
    const float base = ci + (float)iextra;
    DPMARK(1);
    DPCOUNT(4, 1);
    const bool longc = maxlen > (uint32_t)kLongCopy;
    if (__ballot(longc)) {
      if (longc) {
        // forceful long copy (backward-references-hq.ts:518-533): the shortest-distance match
        // longer than kLongCopy; this segment's pending nodes are abandoned and the parse
        // resumes at the copy's end with a new batch
        uint32_t fl = 0, fd = 0;
        float fdc = 0.f;
#pragma unroll
        for (int q = kMaxMatches - 1; q >= 0; q--) {
          if ((uint32_t)q < nm) {
            const uint32_t m = e.m[q];
            if (match_length(m) > (uint32_t)kLongCopy) {
              fd = match_dist(m);
              fl = match_length(m);
              fdc = (float)(e.mc[q] >> 24) * 0.25f;
            }
          }
        }
        const uint32_t limit = b - i;
        if (fl == kMatchLenSat && limit > kMatchLenSat) {
          // a saturated match: measure the copy, kL bytes a step
          GCU8 *cp = (GCU8 *)(data + i), *sp = (GCU8 *)(data + i - fd);
          const uint32_t cap = min(limit, 65535u);
          for (;;) {
            const uint32_t x = fl + hl;
            const uint64_t okb = __ballot(x < cap && cp[x] == sp[x]);
            const uint64_t ok = (okb >> hbase) & kLaneMask;
            if (ok == kLaneMask) {
              fl += kL;
              continue;
            }
            fl += (uint32_t)__ffsll((unsigned long long)~ok) - 1;
            break;
          }
          fl = min(fl, cap);
          if (parts) fl = min(fl, part_cap(abs0 + i, fd, pbits, plag));   // (>= the record's length)
        }
        const int cc = copy_code(fl);
        const bool last = fd == ld;
        const int cmd = combine_codes(ic, cc, last);
        const float fc = base + (float)copy_extra(cc) + cmd_price(cmd, cm) + (last ? (cmd < 128 ? 0.f : dist0) : fdc);
        {
          const uint32_t p = i0 + hl;
          if (p <= i && p != a) choice[gbase + p] = choice_of(chd, chm);
        }
        if (KC) {
          // the ring after the copy (waits for its loads: long copies are rare): node i-1's ring,
          // node i's (its predecessor's, loaded now), fd pushed on it
          const uint32_t r1 = (kf & 3u) ? ring_step(kf & 3u, kp_ld, kp_h, rg) : rg;
          const bool ccopy = !(kf & 4u) && mm >= 2u && (mm >> 16) == 0u;
          const uint32_t hv = ccopy ? ring_hist[hoff + ((i - mm) & (kHistPos - 1)) * 4 + rq] : 0u;
          const uint32_t ri = ring_step(ccopy ? 2u : 1u, ld, hv, r1);
          rg = ring_step(2u, fd, ri, ri);
          kf = 4u;   // (no node i-1, nothing in flight)
        }
        i += fl;
        i0 = i;
        rp_d = 0;
#pragma unroll
        for (int c = 0; c < kC; c++) wc[c] = kInf;
        if (hl == 0) {
          wc[0] = fc;
          wd[0] = fd;
          wm[0] = fl;
        }
        stage();
      }
      wave_sync();
      DPMARK(2);
      continue;
    }
    // the match staircase of i: lengths (clipped) and the packed (distance | cost code) words
    // (both read unconditionally: a masked load would be a branch and a wait per entry)
    const uint32_t actm = 0u - (uint32_t)act;
    uint32_t mL[kMaxMatches], vpk[kMaxMatches];
    if constexpr (kMaxMatches == 4) {
      const uint4 em = *reinterpret_cast<const uint4 *>(e.m), emc = *reinterpret_cast<const uint4 *>(e.mc);
      mL[0] = match_length(em.x) & actm; mL[1] = match_length(em.y) & actm;   // 0 past nm
      mL[2] = match_length(em.z) & actm; mL[3] = match_length(em.w) & actm;
      vpk[0] = emc.x; vpk[1] = emc.y; vpk[2] = emc.z; vpk[3] = emc.w;
    } else {
#pragma unroll
      for (int q = 0; q < kMaxMatches; q++) {
        mL[q] = match_length(e.m[q]) & actm;
        vpk[q] = e.mc[q];
      }
    }
    // the last-distance copy out of node i - 1 (see rp_d): its length R from the loaded bytes
    uint32_t R = 0;
    if (KR) {
      // (at most kRepLen bytes whatever the lanes per segment: a stream's parse must not
      // depend on how many segments share its wave -- a batch encodes each stream as alone)
      const uint64_t eqm = (__ballot(rp_cb == rp_sb) >> hbase) & ((1ull << kRepLen) - 1);
      R = (act && rp_d) ? (eqm == (1ull << kRepLen) - 1 ? (uint32_t)kRepLen : (uint32_t)__ffsll((unsigned long long)~eqm) - 1u) : 0u;
      if (parts && R) R = min(R, part_cap(abs0 + i - 1, rp_d, pbits, plag));
      R = R >= 2 ? R : 0u;
    }
    const uint32_t maxrel = max(max(1u, maxlen), R ? R - 1 : 0u);
    const uint32_t *trow = ptab + ic * kPtabW;

    // relax every edge out of i: lane j of chunk k takes length kL k + j - off
#pragma unroll
    for (int c = 0; c < kC; c++) {
      if (c > 0 && __ballot(act && (uint32_t)(kL * c) <= off + maxrel) == 0) break;
      const uint32_t l = (uint32_t)(kL * c) + hl - off;   // wraps (huge) for consumed nodes
      float cand = kInf;
      uint32_t nd = ld, nmeta = (ins1 << 16) | nx;
      if (l == 1 && act) cand = ci + litcost;
      if (l >= minlen && l <= maxlen) {
        uint32_t x = 0;
#pragma unroll
        for (int q = kMaxMatches - 1; q >= 0; q--)
          x = l <= mL[q] ? vpk[q] : x;   // mL = 0 past nm
        const uint32_t tv = trow[cctab[l]];
        const float pn = (float)__builtin_bit_cast(_Float16, (uint16_t)(tv & 0xFFFF));
        const float pl = (float)__builtin_bit_cast(_Float16, (uint16_t)(tv >> 16));
        nd = match_dist(x);
        if (KD && nd == kCDictMark) nd = min(wabs + i, maxback) + l;   // (d of the copy at i: see kCDictMark)
        const float alt = __builtin_fmaf((float)(x >> 24), 0.25f, pn);   // (exact: code / 4 needs no rounding)
        // a match at the path's last distance is priced with short code 0
        const uint32_t use_last = 0u - (uint32_t)(nd == ld);   // a select, not a branch
        cand = base + __uint_as_float((__float_as_uint(pl) & use_last) | (__float_as_uint(alt) & ~use_last));
        nmeta = l;
      }
      if (cand < wc[c]) {
        wc[c] = cand;
        wd[c] = nd;
        wm[c] = nmeta;
      }
    }
    if (KR && __ballot(R != 0)) {
      // the last-distance copies of lengths 2 .. R <= kRepLen out of node i - 1: lane j of chunk
      // c holds length kL c + j - off + 1 (chunks 0 and 1 hold them all)
      const uint32_t *rrow = ptab + rp_ic * kPtabW;
#pragma unroll
      for (int c = 0; c < 2 && c < kC; c++) {
        const uint32_t lr = (uint32_t)(kL * c) + hl - off + 1u;   // wraps (huge) below the node
        if (lr >= 2u && lr <= R) {
          const uint32_t tv = rrow[cctab[lr]];
          const float cr = rp_base + (float)__builtin_bit_cast(_Float16, (uint16_t)(tv >> 16));
          if (cr < wc[c]) {
            wc[c] = cr;
            wd[c] = rp_d;
            wm[c] = lr;
          }
        }
      }
    }
    // node i's own last-distance candidate: loads now, measured in the next step (a window
    // distance only: not a dictionary word's or a custom-dictionary copy's)
    if (KR) {
      const bool rv = act && use_rep && ins > 0 && ld != 0u && !(words && is_dict(ld)) && ld <= min(wabs + i, maxback);
      rp_d = rv ? ld : 0u;
      rp_base = base;
      rp_ic = (uint32_t)ic;
      rp_cb = 0;
      rp_sb = 1;
      if (rv && hl < (uint32_t)kRepLen && i + hl < b) {
        rp_cb = ((GCU8 *)data)[i + hl];
        rp_sb = ((GCU8 *)data)[(int64_t)(i + hl) - (int64_t)ld];
      }
    }
    DPMARK(3);
    if (KC) {
      // (1) node i-2's candidates (loaded one step ago): the match length over 8 bytes (all 8:
      // the full length where node i-2's staircase holds the same distance -- a cheap 8-byte
      // piece of a longer copy would split it in two commands), and the copies of lengths 4..R
      // relaxed out of node i-2 (lane j of chunk c: length kL c + j + 2 - off)
      const uint32_t x0 = cq_w0 ^ cq_c0, x1 = cq_w1 ^ cq_c1;
      uint32_t R = x0 ? 0u : x1 ? 4u + ((uint32_t)__builtin_ctz(x1) >> 3) : 8u;
      if (__ballot(R == 8u && cq_d != 0u)) {   // (rare: the record is read only then)
        uint32_t full = 0;
#pragma unroll
        for (int q = 0; q < kMaxMatches; q++) full = match_dist(cq_m[q]) == cq_d ? max(full, match_length(cq_m[q])) : full;
        R = R == 8u ? max(R, full) : R;
      }
      R = min(R, cq_lim);
      const bool pass = act && (kf & 8u) && cq_d != 0u && R >= 4u;
      uint64_t pm = __ballot(pass);
      DPCOUNT(2, pm ? 1 : 0);   // (MIB_PROF: steps with a passing candidate; slot 7: the loop's iterations)
      if (pm) {
        // the lengths' copy prices out of node i-2 (its insert code's row), both halves, for the
        // chunks the longest passing candidate reaches: read once, before the candidates' loop
        const uint32_t *crow = ptab + ((kf >> 16) & 0xFFu) * kPtabW;
        // (only the chunks some passing candidate reaches: one ballot a chunk; all kC chunks'
        // lookups unconditionally were 88 of the section's instructions, r06 ISA listing)
        uint32_t ctv[kC];
#pragma unroll
        for (int c = 0; c < kC; c++) {
          ctv[c] = 0u;
          if (c > 1 && __ballot(pass && (uint32_t)(kL * c) + 2u <= off + R) == 0) break;
          const uint32_t lr = (uint32_t)(kL * c) + hl + 2u - off;   // wraps (huge) below node i-2
          if (lr >= 4u && lr <= (uint32_t)kLongCopy) ctv[c] = crow[cctab[lr]];
        }
        // every passing candidate in turn (the lowest short code first), each relaxing lengths
        // 4..R at its own price (the farthest-reaching one alone lost the cheaper short codes of
        // the shorter lengths: records +1.0 % bytes, r06e)
        do {
          const uint32_t mine = (uint32_t)((pm >> hbase) & 0xFFFFull);
          const uint32_t k = mine ? (uint32_t)__builtin_ctz(mine) : 0u;
          const uint32_t src = hbase + k;
          const uint32_t Rk = mine ? bperm(src, R) : 0u, dk = bperm(src, cq_d);
          const float ck = __uint_as_float(bperm(src, __float_as_uint(ccost)));   // short code k's distance symbol
#pragma unroll
          for (int c = 0; c < kC; c++) {
            if (c > 1 && __ballot((uint32_t)(kL * c) + 2u <= off + Rk) == 0) break;
            const uint32_t lr = (uint32_t)(kL * c) + hl + 2u - off;
            if (lr >= 4u && lr <= Rk) {
              const float cr = cq_base + (k ? (float)__builtin_bit_cast(_Float16, (uint16_t)(ctv[c] & 0xFFFF)) + ck
                                            : (float)__builtin_bit_cast(_Float16, (uint16_t)(ctv[c] >> 16)));
              if (cr < wc[c]) {
                wc[c] = cr;
                wd[c] = dk;
                wm[c] = lr;
              }
            }
          }
          pm &= ~__ballot(mine != 0u && hl == k);
          DPCOUNT(7, 1);
        } while (pm);
      }
      DPMARK(6);   // (KC: measuring and relaxing node i-2's candidates)
      // (2) the ring of node i-1, from its edge and the predecessor ring loaded one step ago; kept
      // in the history
      const uint32_t pk = kf & 3u;
      if (pk) {
        rg = ring_step(pk, kp_ld, kp_h, rg);
        ring_hist[hoff + ((i - 1u) & (kHistPos - 1)) * 4 + rq] = rg;
      }
      // (3) node i-1's candidates: a lane per short code, its distance from the ring, its first 8
      // source bytes and node i-1's own loaded below (measured next step)
      bool cv;
      uint32_t cx;
      {
        const uint32_t e0 = quad_entry0(rg), e1 = quad_entry1(rg);
        const uint32_t cb = cj < 4u ? rg : cj < 10u ? e0 : e1;
        const uint32_t cd = cb + (uint32_t)coff;
        const uint32_t x = i - 1u;
        cv = clane && pk != 0u && cb != 0u && !words_on_ring(cb) && cd - 1u < min(x, maxback);
        cq_d = cv ? cd : 0u;
        cx = gbase + x;
        uint32_t cap = b - x;
        if (parts && cv) cap = min(cap, part_cap(abs0 + x, cd, pbits, plag));
        cq_lim = min(cap, (uint32_t)kLongCopy);
        cq_base = kp_base;
      }
      // (4) node i for the next step: its edge, its predecessor's ring (copy edge)
      const bool ccopy = !(kf & 4u) && mm >= 2u && (mm >> 16) == 0u;
      if (act && ccopy) kp_h = ring_hist[hoff + ((i - mm) & (kHistPos - 1)) * 4 + rq];
      kf = (act ? (ccopy ? 2u : 1u) : 0u) | (pk ? 8u : 0u) | ((uint32_t)ic << 8) | (((kf >> 8) & 0xFFu) << 16);
      kp_ld = ld;
      kp_base = base;
      // the candidates' loads last: vmcnt counts loads (and stores) in issue order, so a wait for
      // an older load -- the ring above, KR's bytes -- never waits for these far-back sources
      // (issued before them, KR's measure and the ring step waited out their HBM latency:
      // candidates 1,160 cycles a step, r06r)
      if (cv) {
        cq_w0 = pwords[cx - cq_d];
        cq_w1 = pwords[cx - cq_d + 4u];
        cq_c0 = pwords[cx];
        cq_c1 = pwords[cx + 4u];
        // node i-1's match record (its staircase, as the match finder stored it): the full
        // length of a staircase match at the candidate's distance.  (From its stage entry, while
        // the batch held it, the result depended on where the batches fall -- on the lanes per
        // segment -- and a stream must parse the same in any batch.)
        rec_load(matches + (uint64_t)cx * kMatchRec, cq_m);
      }
    }
    DPMARK(5);   // (KC: the candidates' cycles)
    if (act) i++;
    const bool bend = act && i - i0 == (uint32_t)kL;
    if (__ballot(bend)) {
      // batch end: the window moves down one chunk -- by selects of the whole wave, outside the
      // divergent branch (as moves under the branch, the register allocator copied the window
      // back and forth on every step instead, ~25 moves a step, r05 ISA listing)
#pragma unroll
      for (int c = 0; c + 1 < kC; c++) {
        wc[c] = bend ? wc[c + 1] : wc[c];
        wd[c] = bend ? wd[c + 1] : wd[c];
        wm[c] = bend ? wm[c + 1] : wm[c];
      }
      wc[kC - 1] = bend ? kInf : wc[kC - 1];
      wd[kC - 1] = bend ? 0u : wd[kC - 1];
      wm[kC - 1] = bend ? 0u : wm[kC - 1];
      if (bend) {
        // store the batch's choices, stage the next batch
        if (i0 + hl != a) choice[gbase + i0 + hl] = choice_of(chd, chm);   // node a belongs to the previous segment
        i0 = i;
        stage();
      }
      wave_sync();
    }
    DPMARK(3);
  }
#ifdef MIB_PROF
  if (lane == 0)
    for (int q = 0; q < 8; q++) atomicAdd(&g_dp_prof[q], (unsigned long long)prof[q]);
#endif
}

// ---------------------------------------------------------------- 4. backtrack, wave per segment
// computeShortestPathFromNodes / createCommandsFromPath (backward-references-hq.ts:384-406,
// 610-673) without the distance ring: that is stitched per segment in enc_entropy.hip.
// The path is walked from the segment end in windows of 64 positions: a ballot of the
// window's copy nodes, then a scalar walk that skips each literal run with a bit scan and each
// copy with its length.  The windows are aligned to the segment end and loaded four at a time
// (a chunk of 256 positions), the next chunk in flight while this one is walked; the commands
// gather in lanes (lane k: the k-th of a batch) and are stored 64 at a time.  (A load per
// window issued when the walk reached it, and a store per command from lane 0, left the wave
// waiting on every window: C4 backtrack 2.7 ms a launch.)
constexpr int kBtWin = 4;   // windows per chunk
__global__ __launch_bounds__(64) void backtrack_kernel(const Job *jobs, Seg *segs, int nsegs, const uint64_t *choice,
                                                       RawCmd *raw) {
  const int s = blockIdx.x;
  const int lane = threadIdx.x;
  Seg &sg = segs[s];
  const Job &jb = jobs[sg.job];
  const uint64_t *c = choice + jb.pos_base;
  RawCmd *out = raw + sg.cmd_off;
  const uint32_t a = sg.start;
  const uint32_t cap = (sg.end - a) / 2 + 2;
  uint32_t w = cap;   // commands are written from the end of the slice downward
  uint32_t cur = sg.end, lits = 0, tail = 0;
  bool seen_copy = false;
  uint32_t pend_len = 0, pend_dist = 0, last_dist = 0;
  // the batch of commands in lanes: lane k holds the k-th, stored at w - 1 - k
  uint32_t bi = 0, bl = 0, bd = 0;
  int nb = 0;
  auto put = [&](uint32_t ins, uint32_t len, uint32_t dist) {
    bi = lane == nb ? ins : bi;
    bl = lane == nb ? len : bl;
    bd = lane == nb ? dist : bd;
    if (++nb == 64) {
      RawCmd &o = out[w - 1 - lane];
      o.ins = bi;
      o.len = bl;
      o.dist = bd;
      w -= 64;
      nb = 0;
    }
  };
  auto load_chunk = [&](uint32_t top, uint64_t (&v)[kBtWin]) {   // windows top, top - 64, ...
#pragma unroll
    for (int j = 0; j < kBtWin; j++) {
      const uint32_t p = top - 64u * j - lane;
      v[j] = (top > 64u * j + lane && p > a) ? c[p] : 0ull;
    }
  };
  uint32_t hi = sg.end;   // the chunk's top
  uint64_t va[kBtWin], vb[kBtWin];
  load_chunk(hi, va);
  load_chunk(hi - min(hi, 64u * kBtWin), vb);
  while (cur > a) {
#pragma unroll
    for (int j = 0; j < kBtWin; j++) {
      const uint32_t wtop = hi - 64u * j;
      // (the walk may have jumped past this window, or reached the segment start)
      if (cur > a && cur + 64u > wtop) {
        const uint32_t nvalid = min(64u, wtop - a);
        const uint32_t p = wtop - lane;
        const uint64_t v = va[j];
        uint32_t len = (uint32_t)v;
        if ((uint32_t)lane >= nvalid || len > p - a) len = 0;   // a literal is always a valid edge
        const uint32_t dist = (uint32_t)(v >> 32);
        const uint64_t copies = __ballot(len != 0);
        uint32_t x = wtop - cur;
        for (;;) {
          const uint64_t rest = x < 64 ? (copies >> x) : 0ull;
          const uint32_t y = rest ? x + (uint32_t)(__ffsll((unsigned long long)rest) - 1) : nvalid;
          if (y >= nvalid) {   // literals to the window's end
            lits += nvalid - x;
            cur = wtop - nvalid;
            break;
          }
          lits += y - x;
          const uint32_t L = __builtin_amdgcn_readlane(len, y);
          const uint32_t D = __builtin_amdgcn_readlane(dist, y);
          if (!seen_copy) {
            tail = lits;
            seen_copy = true;
            last_dist = D;
          } else {
            put(lits, pend_len, pend_dist);
          }
          lits = 0;
          pend_len = L;
          pend_dist = D;
          x = y + L;
          if (x >= nvalid) {
            cur = wtop - x;
            break;
          }
        }
      }
    }
    if (cur <= a) break;
    hi -= 64u * kBtWin;
    if (cur + 64u * kBtWin <= hi) {   // a long copy jumped past the next chunk: reload at cur
      hi = sg.end - ((sg.end - cur) / (64u * kBtWin)) * (64u * kBtWin);
      load_chunk(hi, va);
    } else {
#pragma unroll
      for (int j = 0; j < kBtWin; j++) va[j] = vb[j];
    }
    load_chunk(hi - min(hi, 64u * kBtWin), vb);
  }
  if (seen_copy) put(lits, pend_len, pend_dist);
  else tail = lits;
  if (nb) {   // the last, partial batch
    if (lane < nb) {
      RawCmd &o = out[w - 1 - lane];
      o.ins = bi;
      o.len = bl;
      o.dist = bd;
    }
    w -= nb;
  }
  const uint32_t n = cap - w;
  wave_sync();
  // move the commands to the front of the slice; a chunk is read into registers before it
  // is written, and a later chunk's source lies above every earlier chunk's destination
  for (uint32_t q0 = 0; q0 < n; q0 += 64) {
    RawCmd t;
    const uint32_t q = q0 + lane;
    if (q < n) t = out[w + q];
    wave_sync();
    if (q < n) out[q] = t;
    wave_sync();
  }
  if (lane == 0) {
    sg.ncmd = n;
    sg.tail_lits = tail;
    sg.last_dist = last_dist;
  }
}


// ---------------------------------------------------------------- 4b. parse pieces
// The final parse runs on 8 KiB pieces (encode.hip dp_piece_shift: a call with few segments
// leaves SIMDs without a DP wave, and shorter pieces finish a batch's waves more evenly).
// The pieces' commands are then joined per segment: moved to the front of the segment's
// slice, each piece's trailing literals carried into the next piece's first command, as
// carry_kernel does between segments; a copy that ends a piece and one that starts the next
// at the same distance become one copy (a run of zeros stays one command per segment).
// Wave per segment.
__global__ __launch_bounds__(64) void merge_pieces_kernel(const Job *jobs, Seg *segs, const Seg *pieces, RawCmd *raw) {
  Seg &sg = segs[blockIdx.x];
  const Job &jb = jobs[sg.job];
  const int P = 1 << (sg.pieces & 7);
  const Seg *mine = pieces + (sg.pieces >> 3);
  const uint32_t lane = threadIdx.x;
  RawCmd *dst = raw + sg.cmd_off;
  uint32_t n = 0, carry = 0, last = 0;
  for (int k = 0; k < P; k++) {
    const Seg &pc = mine[k];
    const RawCmd *src = raw + pc.cmd_off;   // (at or above dst + n: chunks are read before they are written)
    uint32_t m = pc.ncmd;
    if (m && n && carry == 0) {   // the previous piece ended in a copy: does this one continue it?
      const RawCmd f = src[0], p = dst[n - 1];
      // Never a dictionary copy: a word, or a custom-dictionary tail copy (its distance lies
      // beyond the window at its start, pc.start - p.len: see kCDictMark) -- the copy at the
      // next piece's start with that same distance reads the window (for a tail copy, from
      // stream byte 0), and one joined copy would read past the dictionary's end.
      const uint32_t maxback = (1u << jb.lgwin) - 16;
      const bool p_dict = is_word(jb, p.dist) || (jb.cdict && p.dist > min(jb.win_abs + (pc.start - p.len), maxback));
      if (f.ins == 0 && f.dist == p.dist && !p_dict && !is_word(jb, f.dist)) {
        wave_sync();
        if (lane == 0) dst[n - 1].len = p.len + f.len;
        src++;
        m--;
      }
    }
    for (uint32_t q0 = 0; q0 < m; q0 += 64) {
      const uint32_t q = q0 + lane;
      RawCmd t{0, 0, 0};
      if (q < m) t = src[q];
      wave_sync();
      if (q < m) {
        if (q == 0) t.ins += carry;
        dst[n + q] = t;
      }
      wave_sync();
    }
    if (pc.ncmd) {
      n += m;
      carry = pc.tail_lits;
      last = pc.last_dist;
    } else {
      carry += pc.tail_lits;
    }
  }
  if (lane == 0) {
    sg.ncmd = n;
    sg.tail_lits = carry;
    sg.last_dist = n ? last : 0u;
  }
}
// the sampled copy of the segment table (each segment's first `sample` bytes) and the parse
// pieces (2^ps per segment: kSeg >> ps bytes each, command slices back to back inside the
// segment's, backtrack_kernel's capacity each); thread per segment
__global__ void derive_segs_kernel(const Seg *segs, int nsegs, uint32_t sample, Seg *d_sample, Seg *pieces) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nsegs) return;
  const Seg sg = segs[i];
  if (d_sample) {
    Seg sm = sg;
    sm.end = min(sg.end, sg.start + sample);
    d_sample[i] = sm;
  }
  if (pieces) {
    const int ps = (int)(sg.pieces & 7);
    const uint32_t plen = kSeg >> ps;
    uint32_t off = sg.cmd_off;
    for (int q = 0; q < (1 << ps); q++) {
      Seg pc = sg;
      pc.start = min(sg.end, sg.start + (uint32_t)q * plen);
      pc.end = min(sg.end, pc.start + plen);
      pc.cmd_off = off;
      off += (pc.end - pc.start) / 2 + 2;
      pieces[(sg.pieces >> 3) + q] = pc;
    }
  }
}
void launch_derive_segs(hipStream_t st, const Seg *segs, int nsegs, uint32_t sample, Seg *d_sample, Seg *pieces) {
  if (!d_sample && !pieces) return;
  hipLaunchKernelGGL(derive_segs_kernel, dim3((nsegs + 255) / 256), dim3(256), 0, st, segs, nsegs, sample, d_sample, pieces);
}
void launch_merge_pieces(hipStream_t st, const Job *jobs, Seg *segs, int nsegs, const Seg *pieces, RawCmd *raw) {
  if (nsegs) hipLaunchKernelGGL(merge_pieces_kernel, dim3(nsegs), dim3(64), 0, st, jobs, segs, pieces, raw);
}

// ---------------------------------------------------------------- 5. second-iteration prices
// ZopfliCostModel.setFromCommands + setCostFromHistogram (zopfli-cost-model.ts:68-159):
// histograms of the first parse's literals, command codes and distance codes of a stream
// (block per segment, merged into the stream's histogram), turned into bits per symbol
// (missing symbols: log2 of the sum plus the number of missing symbols, + 2; present ones at
// least 1 bit).  "Last distance" is the parse's notion: the previous copy of the segment.
// A stream's model depends on its own bytes only, so a batch encodes each stream exactly as
// a call of its own does.
constexpr int kHistLen = 256 + 704 + 128;   // literals | commands | distances
// The distance code of a copy at distance d (not a repeat of the last) under a ring r that may
// have unknown (0) entries -- a segment's parse starts without the ring before it: a short code
// 1-15 (as short_code) when d is a known entry or within 3 of entry 0 or 1, else 0.
__device__ __forceinline__ uint32_t known_short_code(uint32_t d, const uint32_t *r) {
  if (r[1] && d == r[1]) return 1;
  if (r[2] && d == r[2]) return 2;
  if (r[3] && d == r[3]) return 3;
  const int64_t a = (int64_t)d - (int64_t)r[0], b = (int64_t)d - (int64_t)r[1];
  if (r[0] && a >= -3 && a <= 3 && a != 0) return a < 0 ? (uint32_t)(4 + 2 * (-a - 1)) : (uint32_t)(5 + 2 * (a - 1));
  if (r[1] && b >= -3 && b <= 3 && b != 0) return b < 0 ? (uint32_t)(10 + 2 * (-b - 1)) : (uint32_t)(11 + 2 * (b - 1));
  return 0;
}
__global__ __launch_bounds__(256) void cmd_stats_kernel(const Job *jobs, const Seg *segs, const RawCmd *raw,
                                                        uint32_t *hist /* kHistLen per job */) {
  __shared__ uint32_t hs[kHistLen], scan[256];
  // the chunk's distances, then their distance codes: the first parse's copies take short codes
  // 1-15 from the distance cache (dp_kernel KC), so the model must see them (setFromCommands
  // counts each command's distance prefix code, zopfli-cost-model.ts:96-110); one thread walks
  // the segment's ring (a sampled first parse: ~200 commands a segment)
  __shared__ uint32_t cdist[256];
  uint32_t ring[4] = {0, 0, 0, 0}, prev_d = 0;
  uint32_t *hl = hs, *hc = hs + 256, *hd = hs + 256 + 704;
  const uint32_t t = threadIdx.x;
  for (uint32_t i = t; i < kHistLen; i += 256) hs[i] = 0;
  __syncthreads();
  const Seg &sg = segs[blockIdx.x];
  const Job &jb = jobs[sg.job];
  const RawCmd *rc = raw + sg.cmd_off;
  const uint32_t n = sg.ncmd;
  uint32_t base = sg.start;
  for (uint32_t q0 = 0; q0 < n; q0 += 256) {
    const uint32_t q = q0 + t;
    RawCmd c{0, 0, 0};
    uint32_t prevd = 0;
    if (q < n) {
      c = rc[q];
      prevd = q ? rc[q - 1].dist : 0u;
    }
    const uint32_t span = c.ins + c.len;
    scan[t] = span;
    __syncthreads();
    for (uint32_t o = 1; o < 256; o <<= 1) {
      const uint32_t v = t >= o ? scan[t - o] : 0u;
      __syncthreads();
      scan[t] += v;
      __syncthreads();
    }
    const uint32_t pos = base + scan[t] - span, tot = scan[255];
    cdist[t] = c.dist;
    __syncthreads();
    if (t == 0 && !jb.binary) {   // (text: explicit codes only, no ring to walk)
      const uint32_t m = min(256u, n - q0);
      for (uint32_t j = 0; j < m; j++) {
        const uint32_t d = cdist[j];
        const bool word = is_word(jb, d);
        uint32_t extra;
        cdist[j] = (!word && d == prev_d) ? 0u : dist_prefix((word ? d & ~kDictFlag : d) + 15, (int)jb.ndirect, (int)jb.npostfix, &extra) & 0x3FFu;
        prev_d = d;
      }
    } else if (t == 0) {
      const uint32_t m = min(256u, n - q0);
      for (uint32_t j = 0; j < m; j++) {
        const uint32_t d = cdist[j];
        const bool word = is_word(jb, d), last = !word && d == prev_d;
        uint32_t code = 0;
        if (!last) {
          // (streams the candidates run in: the short codes they take; others -- text, where the
          // parse offers no short code but the last distance -- price every distance by its
          // explicit code, as before the candidates: C2 0.36352 vs 0.3637 with the short codes)
          const uint32_t sc = (word || !jb.binary) ? 0u : known_short_code(d, ring);
          uint32_t extra;
          code = sc ? sc : dist_prefix((word ? d & ~kDictFlag : d) + 15, (int)jb.ndirect, (int)jb.npostfix, &extra) & 0x3FFu;
          if (!word) {   // every distance code but 0 pushes (a dictionary word: none)
            ring[3] = ring[2];
            ring[2] = ring[1];
            ring[1] = ring[0];
            ring[0] = d;
          }
        }
        prev_d = d;
        cdist[j] = code;
      }
    }
    __syncthreads();
    if (q < n) {
      const bool last = !is_word(jb, c.dist) && c.dist == prevd;
      const int cmd = combine_codes(ins_code(c.ins), copy_code(c.len), last);
      atomicAdd(&hc[cmd], 1u);
      if (cmd >= 128) atomicAdd(&hd[min(cdist[t], 127u)], 1u);
      for (uint32_t j = 0; j < c.ins; j++) atomicAdd(&hl[jb.data[pos + j]], 1u);
    }
    base += tot;
  }
  for (uint32_t p = sg.end - sg.tail_lits + t; p < sg.end; p += 256) atomicAdd(&hl[jb.data[p]], 1u);
  __syncthreads();
  for (uint32_t i = t; i < kHistLen; i += 256)
    if (hs[i]) atomicAdd(&hist[(size_t)sg.job * kHistLen + i], hs[i]);
}
__global__ __launch_bounds__(256) void cost_model_kernel(const uint32_t *hist, CostModel *model) {
  __shared__ uint32_t sums[5];   // literals, commands, distances, missing commands, missing distances
  const uint32_t t = threadIdx.x;
  const uint32_t *hl = hist + (size_t)blockIdx.x * kHistLen, *hc = hl + 256, *hd = hl + 256 + 704;
  if (t < 5) sums[t] = 0;
  __syncthreads();
  {
    uint32_t sc = 0, mc = 0, sd = 0, md = 0;
    for (uint32_t i = t; i < 704; i += 256) {
      sc += hc[i];
      mc += hc[i] == 0;
    }
    if (t < 128) {
      sd = hd[t];
      md = hd[t] == 0;
    }
    atomicAdd(&sums[0], hl[t]);
    atomicAdd(&sums[1], sc);
    atomicAdd(&sums[2], sd);
    atomicAdd(&sums[3], mc);
    atomicAdd(&sums[4], md);
  }
  __syncthreads();
  CostModel &m = model[blockIdx.x];
  auto price = [](uint32_t h, float log2sum, float missing) { return h ? fmaxf(1.f, log2sum - log2f((float)h)) : missing; };
  {
    const float ls = log2f((float)max(sums[0], 1u));
    m.lit[t] = price(hl[t], ls, ls + 2.f);
  }
  {
    const float ls = log2f((float)max(sums[1], 1u)), miss = log2f((float)max(sums[1] + sums[3], 1u)) + 2.f;
    for (uint32_t i = t; i < 704; i += 256) m.cmd[i] = price(hc[i], ls, miss);
  }
  if (t < 128) {
    const float ls = log2f((float)max(sums[2], 1u)), miss = log2f((float)max(sums[2] + sums[4], 1u)) + 2.f;
    m.dist[t] = price(hd[t], ls, miss);
  }
}

// ---------------------------------------------------------------- 6. last-distance copies
// The parse prices a copy at the path's last distance with short code 0, but it only sees the
// distances the match finder offers: the shortest one for each length.  Structured data
// (fonts) repeats records at a fixed stride with a few bytes changed, so the bytes after a
// changed one often match again at the previous copy's distance, for fewer bytes than any
// staircase entry covers -- the reference's parse finds these through its distance-cache
// candidates (backward-references-hq.ts:283-330 / zopfli's "distance cache" loop).  This pass
// walks each command's literal run with the distance of the copy before it (the decoder's
// last distance there): where the run matches at that distance for L >= 2 bytes and the
// stream's cost model (the second iteration's prices) says a code-0 copy of L bytes plus the
// shortened command is cheaper than the literals, the command is split.  A code-0 copy never
// pushes on the distance ring, so every other command's distance code is unchanged.
// Block per segment, thread per command; two sweeps (count, keeping each command's count in
// `cnts`, then rewrite in place from the last chunk down: a command only moves up, past the
// commands split before it; only split commands walk their run again).
constexpr int kRepT = 256;
constexpr int kRepChunks = (int)((kSeg / 2 + 4 + kRepT - 1) / kRepT);
constexpr float kRepMargin = 0.5f;   // bits a split must save
__device__ __forceinline__ float cmd_bits(const CostModel &m, uint32_t ins, int cc, bool last) {
  const int ic = ins_code_sel(ins);
  const int cmd = combine_codes(ic, cc, last);
  return m.cmd[cmd] + (float)ins_extra_sel(ic) + (last && cmd >= 128 ? m.dist[0] : 0.f);
}
// the greedy walk of one literal run [s, e) at distance d: calls out(ins, L) per split, returns
// the literals left before the command's own copy
template <class F>
__device__ __forceinline__ uint32_t rep_walk(const Job &jb, const CostModel &m, uint32_t s, uint32_t e, uint32_t d,
                                             bool skip_first, int cc_k, bool last_k, F out) {
  const uint8_t *data = jb.data;
  uint32_t q = skip_first ? s + 1 : s;
  while (q + 2 <= e) {
    const uint8_t *a = data + q, *b = a - d;
    if (a[0] != b[0] || a[1] != b[1]) {
      q++;
      continue;
    }
    uint32_t L = 2 + match_len(a + 2, b + 2, e - q - 2);
    if (jb.parts) L = min(L, part_cap(jb.abs_base + q, d, jb.part_bits, jb.part_lag));
    if (L >= 2) {
      float lits = 0.f;
      for (uint32_t j = 0; j < L; j++) lits += m.lit[a[j]];
      const int cc = copy_code(L);
      const float before = cmd_bits(m, e - s, cc_k, last_k);
      const float after = cmd_bits(m, q - s, cc, true) + (float)copy_extra(cc) + cmd_bits(m, e - q - L, cc_k, last_k);
      if (lits + before - after > kRepMargin) {
        out(q - s, L);
        s = q + L;
        q = s + 1;   // (byte s mismatches: the copy was measured to its end)
        continue;
      }
    }
    q++;
  }
  return e - s;
}
__global__ __launch_bounds__(kRepT) void rep_kernel(const Job *jobs, Seg *segs, const CostModel *model, RawCmd *raw,
                                                     uint32_t *cnts) {
  typedef hipcub::BlockScan<uint32_t, kRepT> Scan;
  __shared__ typename Scan::TempStorage scan_tmp;
  __shared__ uint32_t chunk_pos[kRepChunks + 1], chunk_split[kRepChunks + 1];
  Seg &sg = segs[blockIdx.x];
  const Job &jb = jobs[sg.job];
  const uint32_t n = sg.ncmd;
  if (jb.uncompressed || n == 0) return;
  const CostModel &m = model[sg.job];
  const uint32_t t = threadIdx.x, nch = (n + kRepT - 1) / kRepT;
  const uint32_t maxback = (1u << jb.lgwin) - 16;
  RawCmd *r = raw + sg.cmd_off;
  // command k: its run [pos, pos + ins), the distance before it, its copy's codes
  // (d: read before any command of the chunk moves)
  auto plan = [&](uint32_t k, const RawCmd &c, uint32_t d, uint32_t pos, auto out) -> uint32_t {
    const uint32_t reach = min(maxback, pos + jb.hist);   // (bytes before data[0]: a streaming chunk's history)
    if (!c.ins || !d || d > reach || is_word(jb, d)) return c.ins;
    return rep_walk(jb, m, pos, pos + c.ins, d, k > 0, copy_code(c.len), c.dist == d, out);
  };
  // sweep 1: positions and split counts per chunk
  uint32_t run = sg.start;
  for (uint32_t ch = 0; ch < nch; ch++) {
    const uint32_t k = ch * kRepT + t;
    RawCmd c{0, 0, 0};
    uint32_t d = 0;
    if (k < n) {
      c = r[k];
      d = k ? r[k - 1].dist : sg.prev_dist;
    }
    uint32_t off, tot;
    Scan(scan_tmp).ExclusiveSum(c.ins + c.len, off, tot);
    __syncthreads();
    uint32_t cnt = 0;
    if (k < n) {
      plan(k, c, d, run + off, [&](uint32_t, uint32_t) { cnt++; });
      cnts[sg.cmd_off + k] = cnt;
    }
    uint32_t coff, ctot;
    Scan(scan_tmp).ExclusiveSum(cnt, coff, ctot);
    __syncthreads();
    if (t == 0) {
      chunk_pos[ch] = run;
      chunk_split[ch] = ctot;
    }
    run += tot;
  }
  __syncthreads();
  if (t == 0) {   // splits before each chunk
    uint32_t acc = 0;
    for (uint32_t ch = 0; ch < nch; ch++) {
      const uint32_t v = chunk_split[ch];
      chunk_split[ch] = acc;
      acc += v;
    }
    chunk_split[nch] = acc;
  }
  __syncthreads();
  if (chunk_split[nch] == 0) return;
  // sweep 2, last chunk first: read the chunk into registers, then write it moved up
  for (int ch = (int)nch - 1; ch >= 0; ch--) {
    const uint32_t k = (uint32_t)ch * kRepT + t;
    RawCmd c{0, 0, 0};
    uint32_t d = 0;
    if (k < n) {
      c = r[k];
      d = k ? r[k - 1].dist : sg.prev_dist;   // (below the chunk, or in it: nothing moved yet)
    }
    uint32_t off, tot;
    Scan(scan_tmp).ExclusiveSum(c.ins + c.len, off, tot);
    __syncthreads();
    const uint32_t cnt = k < n ? cnts[sg.cmd_off + k] : 0u;
    uint32_t coff, ctot;
    Scan(scan_tmp).ExclusiveSum(cnt, coff, ctot);
    __syncthreads();   // (every read of the chunk is done)
    if (k < n) {
      uint32_t w = k + chunk_split[ch] + coff;
      uint32_t left = c.ins;
      if (cnt) left = plan(k, c, d, chunk_pos[ch] + off, [&](uint32_t ins, uint32_t L) { r[w++] = RawCmd{ins, L, d}; });
      r[w] = RawCmd{left, c.len, c.dist};
    }
    __syncthreads();
  }
  if (t == 0) sg.ncmd = n + chunk_split[nch];
}
void launch_rep(hipStream_t st, const Job *jobs, Seg *segs, int nsegs, const CostModel *model, RawCmd *raw, uint32_t *cnts) {
  if (nsegs) hipLaunchKernelGGL(rep_kernel, dim3(nsegs), dim3(kRepT), 0, st, jobs, segs, model, raw, cnts);
}

#ifdef MIB_PROF
extern "C" int mib_debug_read_dp_prof(unsigned long long *out) {
  hipMemcpyFromSymbol(out, HIP_SYMBOL(g_dp_prof), sizeof(unsigned long long) * 8);
  unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  hipMemcpyToSymbol(HIP_SYMBOL(g_dp_prof), z, sizeof(z));
  return 0;
}
#endif
// dp_kernel<4> when there are enough segments for three such waves per SIMD (1024 SIMDs:
// 256 CUs x 4; 143 VGPRs), dp_kernel<2> when there are more than enough for one, else
// dp_kernel<1> (a cadence update()'s 2,048 pieces of 512 B: 390 -> 343 us a chunk with one
// piece a wave, two waves a SIMD, r06 kn_ks).
// Four segments a wave: a step's node fetch, staging and table reads serve four segments and
// text's short staircases still fit 16 lanes' chunks (C4 dp 91.7 -> 75.3 ms, one encode lane,
// r04an; in round 3, before the LDS trim, it was slower: 106.6 -> 119.5 ms)
// FONT mode keeps two: its longer staircases need more of the 16-lane chunks a step (C3 dp
// 38.4 -> 46.6 ms beside the other encode lane, r04ao).
constexpr int kKs4Segs = 3 * 4 * 1024;
static int dp_ks(int nsegs, bool font) {
  static const int v = knob("MIB_DP_KS") ? atoi(knob("MIB_DP_KS")) : 0;   // experiments
  if (v == 1 || v == 2 || v == 4) return v;
  return !font && nsegs >= kKs4Segs ? 4 : nsegs <= 2048 ? 1 : 2;
}
template <bool KD, bool KC>
static void launch_dp_t(hipStream_t st, const Job *jobs, const Seg *segs, int nsegs, const uint32_t *lit_h,
                        const CostModel *model, const uint32_t *matches, uint64_t *choice, bool font,
                        const uint32_t *words, uint32_t *ring_hist, const Mb *mbs, int kc_split) {
  const int ks = dp_ks(nsegs, font), spw = kDpWaves * ks;
  const dim3 g((nsegs + spw - 1) / spw), b(64 * kDpWaves);
  // MIB_CMD_PENALTY (bits, experiment): added to every copy's price, fewer and longer commands
  static const float cmd_pen = knob("MIB_CMD_PENALTY") ? (float)atof(knob("MIB_CMD_PENALTY")) : 0.f;
  // last-distance candidates in the parse: FONT mode (MIB_DP_REP, experiments: 0 off, 2 every mode)
  static const int rep_knob = knob("MIB_DP_REP") ? atoi(knob("MIB_DP_REP")) : 1;
  const bool rep = rep_knob == 2 || (rep_knob == 1 && font);
#define MIB_DP(K, M, R) \
  hipLaunchKernelGGL((dp_kernel<K, M, KD, R, KC>), g, b, 0, st, jobs, segs, nsegs, lit_h, model, matches, choice, cmd_pen, 1, words, ring_hist, mbs, kc_split)
#define MIB_DP_KS(K)                \
  do {                              \
    if (model && rep) MIB_DP(K, true, true);   \
    else if (model) MIB_DP(K, true, false);    \
    else if (rep) MIB_DP(K, false, true);      \
    else MIB_DP(K, false, false);              \
  } while (0)
  if (ks == 1) MIB_DP_KS(1);
  else if (ks == 4) MIB_DP_KS(4);
  else MIB_DP_KS(2);
#undef MIB_DP_KS
#undef MIB_DP
}
// (words, ring_hist: the distance-cache candidates' inputs, dp_ring_hist_bytes; null: none).
// With them, two launches: the candidates' build for the segments whose metablock's literals
// are not UTF-8 text, the plain build for the rest (mbs[].ctx_mode must be set).
void launch_dp(hipStream_t st, const Job *jobs, const Seg *segs, int nsegs, const uint32_t *lit_h, const CostModel *model,
               const uint32_t *matches, uint64_t *choice, bool cdict, bool font, const uint32_t *words, uint32_t *ring_hist,
               const Mb *mbs) {
  const bool kc = words && ring_hist && mbs;
  if (cdict) {
    if (kc) launch_dp_t<true, true>(st, jobs, segs, nsegs, lit_h, model, matches, choice, font, words, ring_hist, mbs, 1);
    launch_dp_t<true, false>(st, jobs, segs, nsegs, lit_h, model, matches, choice, font, words, ring_hist, mbs, kc ? 1 : 0);
  } else {
    if (kc) launch_dp_t<false, true>(st, jobs, segs, nsegs, lit_h, model, matches, choice, font, words, ring_hist, mbs, 1);
    launch_dp_t<false, false>(st, jobs, segs, nsegs, lit_h, model, matches, choice, font, words, ring_hist, mbs, kc ? 1 : 0);
  }
}
size_t dp_ring_hist_bytes(int nsegs) { return (size_t)std::max(nsegs, 1) * kHistPos * 16; }
// words[g] = the four stream bytes at global position g (0 past the stream's end): the
// distance-cache candidates compare 8 bytes with two aligned loads.  Thread per position.
// (only the streams with a metablock the candidates run in: Job.binary)
__global__ void words_kernel(const Job *jobs, const uint32_t *pos_job, const SegRef *seg_ref, uint32_t total, uint32_t *words) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= total || !jobs[pos_job[g >> kSegBits]].binary) return;
  const SegRef r = seg_ref[g >> kSegBits];
  uint32_t v = 0;
#pragma unroll
  for (uint32_t k = 0; k < 4; k++)
    if (g + k < r.end) v |= (uint32_t)r.base[g + k] << (8 * k);
  words[g] = v;
}
// flag = 1 if any stream of the call has a metablock the candidates run in (Job.binary)
__global__ void any_binary_kernel(const Job *jobs, int njobs, uint32_t *flag) {
  uint32_t v = 0;
  for (int j = threadIdx.x; j < njobs; j += blockDim.x) v |= jobs[j].binary;
  if (__syncthreads_or((int)v) && threadIdx.x == 0) *flag = 1u;
  else if (threadIdx.x == 0) *flag = 0u;
}
void launch_any_binary(hipStream_t st, const Job *jobs, int njobs, uint32_t *flag) {
  hipLaunchKernelGGL(any_binary_kernel, dim3(1), dim3(256), 0, st, jobs, njobs, flag);
}
void launch_words(hipStream_t st, const Job *jobs, const uint32_t *pos_job, const SegRef *seg_ref, uint32_t total, uint32_t *words) {
  if (total) hipLaunchKernelGGL(words_kernel, dim3((total + 255) / 256), dim3(256), 0, st, jobs, pos_job, seg_ref, total, words);
}
size_t cost_model_hist_bytes(int njobs) { return (size_t)njobs * kHistLen * 4; }
void launch_cost_model(hipStream_t st, const Job *jobs, int njobs, const Seg *segs, int nsegs, const RawCmd *raw,
                       uint32_t *hist, CostModel *model) {
  hipMemsetAsync(hist, 0, cost_model_hist_bytes(njobs), st);
  hipLaunchKernelGGL(cmd_stats_kernel, dim3(nsegs), dim3(256), 0, st, jobs, segs, raw, hist);
  hipLaunchKernelGGL(cost_model_kernel, dim3(njobs), dim3(256), 0, st, hist, model);
}
void launch_backtrack(hipStream_t st, const Job *jobs, Seg *segs, int nsegs, const uint64_t *choice, RawCmd *raw) {
  hipLaunchKernelGGL(backtrack_kernel, dim3(nsegs), dim3(64), 0, st, jobs, segs, nsegs, choice, raw);
}

}  // namespace enc
}  // namespace mib
