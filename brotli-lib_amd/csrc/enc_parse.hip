// The parse: the wave-per-segment shortest-path DP and the
// backtrack that turns its choices into commands.
#include "enc_common.h"

namespace mib {
namespace enc {

// ---------------------------------------------------------------- 3. DP parse, wave per segment
// Shortest path over positions (updateNodes / computeShortestPathFromNodes,
// backward-references-hq.ts:267-406): node i holds the cheapest cost of reaching i, the
// insert length since the last copy, and the path's last distance.  Edges: one literal;
// the staircase matches of i (lanes relax consecutive lengths in parallel); a copy at the
// path's last distance (short code 0).  A match longer than kLongCopy is taken outright and
// the parse jumps to its end, as the reference does (:518-533).
//
// Everything a position needs that does not depend on the DP state (its matches, its
// literal byte, the bytes ahead) is staged into LDS 64 positions at a time with coalesced
// loads; the only load left inside the serial loop is the 64-byte window at the path's
// last distance, issued before the relaxations that hide it.
constexpr int kBatch = 64;
constexpr float kInf = 3.0e38f;
constexpr int kChunks = (kLongCopy + 64) / 64;   // length chunks of 64 lanes covering 0..kLongCopy

// node meta: last distance (32) | copy length that reached it (16, 0 = literal) | insert length (16)
__device__ __forceinline__ uint64_t pack_node(uint32_t ld, uint32_t clen, uint32_t ins) {
  return (uint64_t)ld | ((uint64_t)clen << 32) | ((uint64_t)min(ins, 65535u) << 48);
}
__device__ __forceinline__ uint64_t node_choice(uint64_t m) {   // (distance << 32) | length, 0 = literal
  uint32_t cl = (uint32_t)(m >> 32) & 0xFFFF;
  return cl ? (((uint64_t)(uint32_t)m << 32) | cl) : 0ull;
}

__global__ __launch_bounds__(64) void dp_kernel(const Job *jobs, const Seg *segs, const uint32_t *lit_histo,
                                                const uint64_t *matches, const uint8_t *nmatch,
                                                uint64_t *choice /* per position+1 */) {
  __shared__ float cost[kRing];
  __shared__ uint64_t meta[kRing];
  __shared__ float cmdc[704];
  __shared__ float distc[128];
  __shared__ float litc[256];
  __shared__ float blit[kBatch];                   // literal cost of each batch position
  __shared__ uint8_t bnm[kBatch];
  __shared__ uint64_t bmt[kBatch * kMaxMatches];   // (distance << 32) | length
  __shared__ float bmc[kBatch * kMaxMatches];      // distance symbol cost + extra bits
  const int lane = threadIdx.x;
  const Seg sg = segs[blockIdx.x];
  const Job &jb = jobs[sg.job];
  const uint8_t *data = jb.data;
  // cost model: literals from the stream's order-0 histogram (zopfli-cost-model.ts:163-189),
  // commands / distances from the reference's first-iteration heuristic (:54-64).
  {
    uint32_t total = 0;
    for (int i = 0; i < 256; i++) total += lit_histo[sg.job * 256 + i];
    float lt = log2f((float)max(total, 1u));
    for (int i = lane; i < 256; i += 64) {
      uint32_t c = lit_histo[sg.job * 256 + i];
      float v = c ? lt - log2f((float)c) : lt + 2.f;
      litc[i] = v < 1.f ? 1.f : v;
    }
    for (int i = lane; i < 704; i += 64) cmdc[i] = log2f(11.f + i);
    for (int i = lane; i < 128; i += 64) distc[i] = log2f(20.f + i);
  }
  for (int i = lane; i < kRing; i += 64) {
    cost[i] = kInf;
    meta[i] = 0;
  }
  // copy code / extra bits of the lengths this lane relaxes (l = 64 k + lane)
  int ccl[kChunks];
  float cxl[kChunks];
#pragma unroll
  for (int k = 0; k < kChunks; k++) {
    uint32_t l = max(2u, (uint32_t)(64 * k + lane));
    ccl[k] = copy_code(l);
    cxl[k] = (float)kCopyExtra[ccl[k]];
  }
  // command cost per lane length for the current insert code: explicit distance / last distance
  float cm[kChunks], cml[kChunks];
  int cached_ic = -1;
  wave_sync();
  const uint32_t a = sg.start, b = sg.end;
  const uint32_t gbase = jb.pos_base;
  if (lane == 0) cost[a % kRing] = 0.f;
  // the path's last distance: verified run [c_from, c_upto) of data[p] == data[p - c_ld]
  uint32_t c_ld = 0, c_from = 0, c_upto = 0;
  bool c_end = false;   // c_upto is a mismatch (or the segment end), not just "verified so far"
  uint32_t i = a;
  while (i < b) {
    // ---- stage the next batch: matches and their distance costs, literal costs
    const uint32_t i0 = i;
    const uint32_t nb = min((uint32_t)kBatch, b - i0);
    wave_sync();
    {
      int nm = 0;
      if ((uint32_t)lane < nb) {
        nm = nmatch[gbase + i0 + lane];
        blit[lane] = litc[data[i0 + lane]];
      }
      bnm[lane] = (uint8_t)nm;
      const uint64_t *src = matches + (uint64_t)(gbase + i0 + lane) * kMaxMatches;
      for (int q = 0; q < nm; q++) {
        uint64_t m = src[q];
        uint32_t extra;
        uint32_t dp = dist_prefix((uint32_t)(m >> 32) + 15, (int)jb.ndirect, (int)jb.npostfix, &extra);
        bmt[lane * kMaxMatches + q] = m;
        bmc[lane * kMaxMatches + q] = (float)(dp >> 10) + distc[min(dp & 0x3FFu, 127u)];
      }
    }
    wave_sync();
    bool forced = false;
    while (i < i0 + nb) {
      const int slot = i % kRing;
      const float ci = cost[slot];
      const uint64_t mi = meta[slot];
      const uint32_t ld = (uint32_t)mi, ins_i = (uint32_t)(mi >> 48);
      const uint32_t off = i - i0;
      const uint32_t limit = b - i;
      const float litcost = blit[off];
      // the staircase of (distance, length), clipped at the segment end
      const int nm = bnm[off];
      uint32_t md[kMaxMatches], mL[kMaxMatches];
      float mc[kMaxMatches];
#pragma unroll
      for (int q = 0; q < kMaxMatches; q++) {
        const uint64_t m = q < nm ? bmt[off * kMaxMatches + q] : 0ull;
        md[q] = (uint32_t)(m >> 32);
        mL[q] = min((uint32_t)m, limit);
        mc[q] = q < nm ? bmc[off * kMaxMatches + q] : 0.f;
      }
      wave_sync();
      if (lane == 0) cost[slot] = kInf;   // the slot now serves position i + kRing
      // ---- run length at the path's last distance (short code 0), from the cache
      uint32_t ldlen = 0;
      if (ld != 0 && ld <= i) {
        if (!(ld == c_ld && i >= c_from && i <= c_upto)) {
          c_ld = ld;
          c_from = c_upto = i;
          c_end = false;
        }
        while (!c_end && c_upto - i <= (uint32_t)kLongCopy) {
          const uint32_t k = c_upto + lane;
          const bool eq = k < b && data[k] == data[k - ld];
          const uint64_t ok = __ballot(eq);
          if (ok == ~0ull) {
            c_upto += 64;
          } else {
            c_upto += __ffsll((unsigned long long)~ok) - 1;
            c_end = true;
          }
        }
        ldlen = min(c_upto - i, limit);
      }
      const int ic = ins_code(ins_i);
      const float base = ci + (float)kInsExtra[ic];
      // ---- forceful long copy (backward-references-hq.ts:518-533)
      uint32_t fd = 0, fl = 0;
      float fc = 0.f;
      if (ldlen > (uint32_t)kLongCopy) {
        while (!c_end && c_upto - i < 65535u) {   // take the whole run
          const uint32_t k = c_upto + lane;
          const bool eq = k < b && data[k] == data[k - ld];
          const uint64_t ok = __ballot(eq);
          if (ok == ~0ull) {
            c_upto += 64;
          } else {
            c_upto += __ffsll((unsigned long long)~ok) - 1;
            c_end = true;
          }
        }
        fl = min(min(c_upto - i, limit), 65535u);
        fd = ld;
        const int cc = copy_code(fl);
        const int cmd = combine_codes(ic, cc, true);
        fc = base + (float)kCopyExtra[cc] + cmdc[cmd] + (cmd < 128 ? 0.f : distc[0]);
      } else {
#pragma unroll
        for (int q = 0; q < kMaxMatches; q++) {
          if (!fl && q < nm && mL[q] > (uint32_t)kLongCopy) {
            fd = md[q];
            fl = mL[q];
            const int cc = copy_code(fl);
            fc = base + mc[q] + (float)kCopyExtra[cc] + cmdc[combine_codes(ic, cc, false)];
          }
        }
      }
      if (fl) {
        // flush the batch's finished nodes, abandon every pending node, resume at the end
        for (uint32_t p = i0 + lane; p <= i; p += 64)
          if (p != a) choice[gbase + p] = node_choice(meta[p % kRing]);
        wave_sync();
        for (int t = lane; t < kRing; t += 64) cost[t] = kInf;
        wave_sync();
        const uint32_t skip_to = i + fl;
        if (lane == 0) {
          cost[skip_to % kRing] = fc;
          meta[skip_to % kRing] = pack_node(fd, fl, 0);
        }
        wave_sync();
        i = skip_to;
        forced = true;
        break;
      }
      if (ic != cached_ic) {
        cached_ic = ic;
#pragma unroll
        for (int k = 0; k < kChunks; k++) {
          cm[k] = cxl[k] + cmdc[combine_codes(ic, ccl[k], false)];
          const int cmd = combine_codes(ic, ccl[k], true);
          cml[k] = cxl[k] + cmdc[cmd] + (cmd < 128 ? 0.f : distc[0]);
        }
      }
      // ---- relax every edge out of i: lane l of chunk k takes length 64 k + l, choosing
      // the literal (l = 1), the shortest-distance match covering l, or the last distance
      uint32_t maxlen = 1;
#pragma unroll
      for (int q = 0; q < kMaxMatches; q++)
        if (q < nm) maxlen = max(maxlen, mL[q]);
      maxlen = max(maxlen, ldlen);
#pragma unroll
      for (int k = 0; k < kChunks; k++) {
        if (64 * k > (int)maxlen) break;
        const uint32_t l = 64 * k + lane;
        float best = kInf;
        uint64_t bm = 0;
        if (l == 1) {
          best = ci + litcost;
          bm = pack_node(ld, 0, ins_i + 1);
        } else if (l >= 2 && l <= maxlen) {
          if (l >= 4) {
            bool found = false;
#pragma unroll
            for (int q = 0; q < kMaxMatches; q++) {
              if (!found && q < nm && mL[q] >= l) {
                found = true;
                best = base + mc[q] + cm[k];
                bm = pack_node(md[q], l, 0);
              }
            }
          }
          if (l <= ldlen) {
            const float c2 = base + cml[k];
            if (c2 < best) {
              best = c2;
              bm = pack_node(ld, l, 0);
            }
          }
        }
        if (best < kInf) {
          const int ts = (i + l) % kRing;
          if (best < cost[ts]) {
            cost[ts] = best;
            meta[ts] = bm;
          }
        }
      }
      wave_sync();
      i++;
    }
    if (!forced) {   // the batch's nodes are final: one coalesced store of their choices
      const uint32_t p = i0 + lane;
      if ((uint32_t)lane < nb && p != a) choice[gbase + p] = node_choice(meta[p % kRing]);
    }
  }
  // the segment's end node
  if (lane == 0) choice[gbase + b] = node_choice(meta[b % kRing]);
}

// ---------------------------------------------------------------- 4. backtrack, lane per segment
// computeShortestPathFromNodes / createCommandsFromPath (backward-references-hq.ts:384-406,
// 610-673) without the distance ring: that is stitched per segment in enc_entropy.hip.
__global__ void backtrack_kernel(const Job *jobs, Seg *segs, int nsegs, const uint64_t *choice, RawCmd *raw) {
  int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= nsegs) return;
  Seg &sg = segs[s];
  const Job &jb = jobs[sg.job];
  const uint64_t *c = choice + jb.pos_base;
  RawCmd *out = raw + sg.cmd_off;
  // walk back, writing commands from the end of the slice downward
  uint32_t cap = (sg.end - sg.start) / 2 + 2;
  uint32_t w = cap;
  uint32_t p = sg.end, lits = 0, tail = 0;
  bool seen_copy = false;
  uint32_t pend_len = 0, pend_dist = 0, last_dist = 0;
  while (p > sg.start) {
    uint64_t v = c[p];
    uint32_t len = (uint32_t)v;
    if (len > p - sg.start) len = 0;   // never taken; a literal is always a valid edge
    if (len == 0) {
      lits++;
      p--;
      continue;
    }
    if (!seen_copy) {
      tail = lits;
      seen_copy = true;
      last_dist = (uint32_t)(v >> 32);
    } else {
      w--;
      out[w].ins = lits;
      out[w].len = pend_len;
      out[w].dist = pend_dist;
    }
    lits = 0;
    pend_len = len;
    pend_dist = (uint32_t)(v >> 32);
    p -= len;
  }
  if (seen_copy) {
    w--;
    out[w].ins = lits;
    out[w].len = pend_len;
    out[w].dist = pend_dist;
  } else {
    tail = lits;
  }
  uint32_t n = cap - w;
  for (uint32_t q = 0; q < n; q++) out[q] = out[w + q];
  sg.ncmd = n;
  sg.tail_lits = tail;
  sg.last_dist = last_dist;
}


void launch_dp(hipStream_t st, const Job *jobs, const Seg *segs, int nsegs, const uint32_t *lit_h,
               const uint64_t *matches, const uint8_t *nmatch, uint64_t *choice) {
  hipLaunchKernelGGL(dp_kernel, dim3(nsegs), dim3(64), 0, st, jobs, segs, lit_h, matches, nmatch, choice);
}
void launch_backtrack(hipStream_t st, const Job *jobs, Seg *segs, int nsegs, const uint64_t *choice, RawCmd *raw) {
  hipLaunchKernelGGL(backtrack_kernel, dim3((nsegs + 63) / 64), dim3(64), 0, st, jobs, segs, nsegs, choice, raw);
}

}  // namespace enc
}  // namespace mib
