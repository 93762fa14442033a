// The parse: the wave-per-segment shortest-path DP and the
// backtrack that turns its choices into commands.
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
// One wave runs kG = 2 segments side by side, 32 lanes each: per step every group advances
// its own segment by one position, its 32 lanes relaxing 32 copy lengths at a time, so the
// per-position bookkeeping is paid once per 2 positions.  (Measured on MI355X, 1 GiB of
// text: 1 x 64 lanes 696 ms, 2 x 32 474 ms, 4 x 16 518 ms, 8 x 8 897 ms -- beyond two
// groups the groups' divergent refills and long-match chunks cost more than they save.)
// Everything a position needs (its matches with their distance costs, its literal cost) is
// staged into LDS kBatch positions at a time from registers that were loaded one batch
// ahead, so the serial loop itself never waits on global memory.
constexpr int kGL = 32;        // lanes per segment
constexpr int kG = 64 / kGL;   // segments per wave
constexpr int kBatch = kGL;    // positions staged per refill (one per lane)
constexpr int kCache = kGL >= 32 ? 1 : 32 / kGL;   // length chunks whose command costs stay in registers
constexpr uint32_t kRingMask = kRing - 1;
constexpr float kInf = 3.0e38f;
static_assert(kLongCopy + kBatch < kRing, "a batch's nodes must survive until they are flushed");

// node meta: last distance (32) | copy length that reached it (16, 0 = literal) | insert length (16)
__device__ __forceinline__ uint64_t pack_node(uint32_t ld, uint32_t clen, uint32_t ins) {
  return (uint64_t)ld | ((uint64_t)clen << 32) | ((uint64_t)min(ins, 65535u) << 48);
}
__device__ __forceinline__ uint64_t node_choice(uint64_t m) {   // (distance << 32) | length, 0 = literal
  uint32_t cl = (uint32_t)(m >> 32) & 0xFFFF;
  return cl ? (((uint64_t)(uint32_t)m << 32) | cl) : 0ull;
}

struct Staged {   // one position's parse inputs, loaded ahead
  uint32_t m[kMaxMatches];
  uint32_t nm;
  uint32_t lit;
};
__device__ __forceinline__ void load_staged(Staged &st, const uint32_t *matches, const uint8_t *nmatch, const uint8_t *data,
                                            uint32_t g, uint32_t p) {
  st.nm = nmatch[g];
  st.lit = data[p];
  const uint32_t *src = matches + (uint64_t)g * kMaxMatches;
#pragma unroll
  for (int q = 0; q < kMaxMatches; q++) st.m[q] = src[q];   // entries past nm are ignored
}

__global__ __launch_bounds__(64) void dp_kernel(const Job *jobs, const Seg *segs, int nsegs, const uint32_t *lit_histo,
                                                const uint32_t *matches, const uint8_t *nmatch,
                                                uint64_t *choice /* per position+1 */) {
  // per-group rows are padded so the 4 groups' same-offset accesses fall in different banks
  __shared__ float cost[kG][kRing + 1];
  __shared__ uint64_t meta[kG][kRing + 1];
  __shared__ uint16_t litc[kG][256 + 2];   // literal cost x 256
  __shared__ float cmdc[704];
  __shared__ float distc[128];
  __shared__ float blit[kG][kBatch + 1];
  __shared__ uint8_t bnm[kG][kBatch + 4];
  __shared__ uint32_t bmt[kG][kBatch * kMaxMatches + 1];   // pack_match(distance, length)
  __shared__ float bmc[kG][kBatch * kMaxMatches + 1];      // distance symbol cost + extra bits
  const int lane = threadIdx.x, g = lane / kGL, sl = lane % kGL;
  const int s = blockIdx.x * kG + g;
  const bool valid = s < nsegs;
  const Seg sg = segs[valid ? s : 0];
  const Job &jb = jobs[sg.job];
  const uint8_t *data = jb.data;
  const uint32_t a = sg.start, b = sg.end, gbase = jb.pos_base;
  for (int i = lane; i < 704; i += 64) cmdc[i] = log2f(11.f + i);
  for (int i = lane; i < 128; i += 64) distc[i] = log2f(20.f + i);
  // literal costs from the stream's order-0 histogram (zopfli-cost-model.ts:163-189)
  {
    uint32_t part = 0;
    for (int i = sl; i < 256; i += kGL) part += lit_histo[sg.job * 256 + i];
    for (int o = kGL / 2; o; o >>= 1) part += __shfl_xor(part, o, kGL);
    const float lt = log2f((float)max(part, 1u));
    for (int i = sl; i < 256; i += kGL) {
      const uint32_t c = lit_histo[sg.job * 256 + i];
      const float v = c ? lt - log2f((float)c) : lt + 2.f;
      litc[g][i] = (uint16_t)(fminf(fmaxf(v, 1.f), 255.f) * 256.f);
    }
  }
  for (int i = sl; i < kRing; i += kGL) {
    cost[g][i] = kInf;
    meta[g][i] = 0;
  }
  wave_sync();
  if (sl == 0) cost[g][a & kRingMask] = 0.f;
  // command cost of this lane's lengths in chunks 0 and 1 for the current insert code
  int ccA[kCache];
  float cmA[kCache], cmlA[kCache];
#pragma unroll
  for (int c = 0; c < kCache; c++) {
    ccA[c] = copy_code(max(2u, (uint32_t)(kGL * c + sl)));
    cmA[c] = cmlA[c] = 0.f;
  }
  int cached_ic = -1;
  bool active = valid && a < b;
  uint32_t i = a, i0 = a, nb = 0;
  bool flushed = true;   // the current batch's choices are already stored
  // the batch after the current one, in registers
  Staged pf;
  uint32_t pf_at = 0xFFFFFFFFu;
  if (active && a + sl < b) {
    load_staged(pf, matches, nmatch, data, gbase + a + sl, a + sl);
    pf_at = a;
  }
  wave_sync();
  for (;;) {
    // ---- per group: finish a batch (store its choices), finish the segment, or stage
    if (active && i >= i0 + nb) {
      if (!flushed && (uint32_t)sl < nb && i0 + sl != a) choice[gbase + i0 + sl] = node_choice(meta[g][(i0 + sl) & kRingMask]);
      if (i >= b) {
        if (sl == 0) choice[gbase + b] = node_choice(meta[g][b & kRingMask]);
        active = false;
      } else {
        i0 = i;
        nb = min((uint32_t)kBatch, b - i0);
        flushed = false;
        Staged cur;
        if (pf_at == i0) {
          cur = pf;
        } else if (i0 + sl < b) {   // the parse jumped past the prefetched batch
          load_staged(cur, matches, nmatch, data, gbase + i0 + sl, i0 + sl);
        }
        // prefetch the next batch
        const uint32_t nx = i0 + nb;
        if (nx + sl < b) load_staged(pf, matches, nmatch, data, gbase + nx + sl, nx + sl);
        pf_at = nx;
        int nm = 0;
        if ((uint32_t)sl < nb) {
          nm = (int)cur.nm;
          blit[g][sl] = (float)litc[g][cur.lit] * (1.f / 256.f);
        }
        bnm[g][sl] = (uint8_t)nm;
#pragma unroll
        for (int q = 0; q < kMaxMatches; q++) {
          if (q < nm) {
            const uint32_t m = cur.m[q];
            uint32_t extra;
            const uint32_t dp = dist_prefix(match_dist(m) + 15, (int)jb.ndirect, (int)jb.npostfix, &extra);
            bmt[g][sl * kMaxMatches + q] = m;
            bmc[g][sl * kMaxMatches + q] = (float)(dp >> 10) + distc[min(dp & 0x3FFu, 127u)];
          }
        }
      }
    }
    wave_sync();
    if (!__ballot(active)) break;
    if (!active) continue;
    // ---- one position per group
    const uint32_t slot = i & kRingMask;
    const float ci = cost[g][slot];
    const uint64_t mi = meta[g][slot];
    const uint32_t ld = (uint32_t)mi, ins_i = (uint32_t)(mi >> 48);
    const uint32_t off = i - i0, limit = b - i;
    const float litcost = blit[g][off];
    const int nm = bnm[g][off];
    uint32_t md[kMaxMatches], mL[kMaxMatches];
    float mc[kMaxMatches];
#pragma unroll
    for (int q = 0; q < kMaxMatches; q++) {
      const uint32_t m = q < nm ? bmt[g][off * kMaxMatches + q] : 0u;
      md[q] = match_dist(m);
      mL[q] = min(match_length(m), limit);
      mc[q] = q < nm ? bmc[g][off * kMaxMatches + q] : 0.f;
    }
    wave_sync();
    if (sl == 0) cost[g][slot] = kInf;   // the slot now serves position i + kRing
    const int ic = ins_code(ins_i);
    const float base = ci + (float)kInsExtra[ic];
    if (ic != cached_ic) {
      cached_ic = ic;
#pragma unroll
      for (int c = 0; c < kCache; c++) {
        cmA[c] = (float)kCopyExtra[ccA[c]] + cmdc[combine_codes(ic, ccA[c], false)];
        const int cmd = combine_codes(ic, ccA[c], true);
        cmlA[c] = (float)kCopyExtra[ccA[c]] + cmdc[cmd] + (cmd < 128 ? 0.f : distc[0]);
      }
    }
    // forceful long copy (backward-references-hq.ts:518-533)
    uint32_t fl = 0, fd = 0;
    float fc = 0.f;
#pragma unroll
    for (int q = 0; q < kMaxMatches; q++) {
      if (!fl && q < nm && mL[q] > (uint32_t)kLongCopy) {
        fd = md[q];
        fl = mL[q];
        const int cc = copy_code(fl);
        const bool last = fd == ld;
        const int cmd = combine_codes(ic, cc, last);
        fc = base + (float)kCopyExtra[cc] + cmdc[cmd] + (last ? (cmd < 128 ? 0.f : distc[0]) : mc[q]);
      }
    }
    if (fl == kMatchLenSat && limit > kMatchLenSat) {
      // a saturated match: measure the copy (the group's lanes compare kGL bytes a step)
      const uint8_t *cur = data + i, *src = data + i - fd;
      const uint32_t cap = min(limit, 65535u);
      for (;;) {
        const uint32_t x = fl + sl;
        const bool eq = x < cap && cur[x] == src[x];
        const uint64_t ok = (__ballot(eq) >> (kGL * g)) & ((kGL == 64) ? ~0ull : ((1ull << kGL) - 1));
        if (ok == ((kGL == 64) ? ~0ull : ((1ull << kGL) - 1))) {
          fl += kGL;
          continue;
        }
        fl += __ffsll((unsigned long long)~ok) - 1;
        break;
      }
      fl = min(fl, cap);
      const int cc = copy_code(fl);
      const bool last = fd == ld;
      const int cmd = combine_codes(ic, cc, last);
      float dc = 0.f;
#pragma unroll
      for (int q = 0; q < kMaxMatches; q++)
        if (q < nm && md[q] == fd) dc = mc[q];
      fc = base + (float)kCopyExtra[cc] + cmdc[cmd] + (last ? (cmd < 128 ? 0.f : distc[0]) : dc);
    }
    if (fl) {
      // store the batch's finished nodes, abandon every pending node, resume at the copy's end
      for (uint32_t p = i0 + sl; p <= i; p += kGL)
        if (p != a) choice[gbase + p] = node_choice(meta[g][p & kRingMask]);
      wave_sync();
      for (int t = sl; t < kRing; t += kGL) cost[g][t] = kInf;
      wave_sync();
      i += fl;
      if (sl == 0) {
        cost[g][i & kRingMask] = fc;
        meta[g][i & kRingMask] = pack_node(fd, fl, 0);
      }
      flushed = true;
      nb = 0;
      i0 = i;
      continue;
    }
    // relax every edge out of i: lane sl of chunk k takes length kGL k + sl, choosing the
    // literal (length 1) or the shortest-distance match covering it
    uint32_t maxlen = 1;
#pragma unroll
    for (int q = 0; q < kMaxMatches; q++)
      if (q < nm) maxlen = max(maxlen, mL[q]);
    for (uint32_t k = 0; kGL * k <= maxlen; k++) {
      const uint32_t l = kGL * k + sl;
      float best = kInf;
      uint64_t bm = 0;
      if (l == 1) {
        best = ci + litcost;
        bm = pack_node(ld, 0, ins_i + 1);
      } else if (l >= 4 && l <= maxlen) {
        float cmx = 0.f, cml = 0.f;
        bool cached = false;
#pragma unroll
        for (int c = 0; c < kCache; c++)
          if (k == (uint32_t)c) {
            cmx = cmA[c];
            cml = cmlA[c];
            cached = true;
          }
        if (!cached) {
          const int cc = copy_code(l);
          const int cmd = combine_codes(ic, cc, true);
          cmx = (float)kCopyExtra[cc] + cmdc[combine_codes(ic, cc, false)];
          cml = (float)kCopyExtra[cc] + cmdc[cmd] + (cmd < 128 ? 0.f : distc[0]);
        }
        bool found = false;
#pragma unroll
        for (int q = 0; q < kMaxMatches; q++) {
          if (!found && q < nm && mL[q] >= l) {
            found = true;
            best = base + (md[q] == ld ? cml : mc[q] + cmx);
            bm = pack_node(md[q], l, 0);
          }
        }
      }
      if (best < kInf) {
        const uint32_t ts = (i + l) & kRingMask;
        if (best < cost[g][ts]) {
          cost[g][ts] = best;
          meta[g][ts] = bm;
        }
      }
    }
    i++;
  }
}

// ---------------------------------------------------------------- 4. backtrack, wave per segment
// computeShortestPathFromNodes / createCommandsFromPath (backward-references-hq.ts:384-406,
// 610-673) without the distance ring: that is stitched per segment in enc_entropy.hip.
// The path is walked from the segment end in windows of 64 positions: one coalesced load
// of the window's choices, a ballot of its copy nodes, then a scalar walk that skips each
// literal run with a bit scan and each copy with its length.
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
  while (cur > a) {
    const uint32_t nvalid = min(64u, cur - a);
    const uint32_t p = cur - lane;
    uint64_t v = 0;
    if ((uint32_t)lane < nvalid) v = c[p];
    uint32_t len = (uint32_t)v;
    if ((uint32_t)lane >= nvalid || len > p - a) len = 0;   // a literal is always a valid edge
    const uint32_t dist = (uint32_t)(v >> 32);
    const uint64_t copies = __ballot(len != 0);
    uint32_t x = 0;
    for (;;) {
      const uint64_t rest = x < 64 ? (copies >> x) : 0ull;
      const uint32_t y = rest ? x + (uint32_t)(__ffsll((unsigned long long)rest) - 1) : nvalid;
      if (y >= nvalid) {   // literals to the window's end
        lits += nvalid - x;
        cur -= nvalid;
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
        w--;
        if (lane == 0) {
          out[w].ins = lits;
          out[w].len = pend_len;
          out[w].dist = pend_dist;
        }
      }
      lits = 0;
      pend_len = L;
      pend_dist = D;
      x = y + L;
      if (x >= nvalid) {
        cur -= x;
        break;
      }
    }
  }
  if (seen_copy) {
    if (lane == 0) {
      out[w - 1].ins = lits;
      out[w - 1].len = pend_len;
      out[w - 1].dist = pend_dist;
    }
    w--;
  } else {
    tail = lits;
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


void launch_dp(hipStream_t st, const Job *jobs, const Seg *segs, int nsegs, const uint32_t *lit_h,
               const uint32_t *matches, const uint8_t *nmatch, uint64_t *choice) {
  hipLaunchKernelGGL(dp_kernel, dim3((nsegs + kG - 1) / kG), dim3(64), 0, st, jobs, segs, nsegs, lit_h, matches, nmatch,
                     choice);
}
void launch_backtrack(hipStream_t st, const Job *jobs, Seg *segs, int nsegs, const uint64_t *choice, RawCmd *raw) {
  hipLaunchKernelGGL(backtrack_kernel, dim3(nsegs), dim3(64), 0, st, jobs, segs, nsegs, choice, raw);
}

}  // namespace enc
}  // namespace mib
