// Match finding: the LDS-tiled candidate walk over each stream's
// hash buckets (laid out as flat chains by the bucket sort, enc_sort.hip).
#include <algorithm>
#include <cstdlib>

#include "enc_common.h"

namespace mib {
namespace enc {

// ---------------------------------------------------------------- 2. matches
// One thread per SORTED entry: a bucket is a run of equal keys with positions ascending, so
// the candidates of entry r are entries r-1, r-2, ... (most recent first) -- the
// reference's hash chain / tree candidates (hash-binary-tree.ts:156-227), depth by
// quality.  A 256-entry tile plus the 64 entries before it is staged in LDS with the 32
// bytes following each position, so candidates are rejected or measured without touching
// HBM unless a match reaches 32 bytes; only such matches extend through global memory.  The
// staircase of strictly increasing lengths (shortest distance for each length) is kept,
// longest last.
constexpr int kBack = 64;
constexpr int kPreW = 4;   // staged prefix: 4 x 8 bytes

// 32 bytes at p as four little-endian 64-bit words (zero past avail)
__device__ __forceinline__ void load_prefix32(const uint8_t *p, uint32_t avail, uint64_t *o) {
  if (avail >= 36) {   // nine aligned words (all inside the stream) and funnel shifts
    const uintptr_t a = (uintptr_t)p;
    // (global, not flat: the stream bytes are device memory; a flat load also counts on lgkmcnt)
    typedef const __attribute__((address_space(1))) uint32_t GU32;
    GU32 *w = (GU32 *)(a & ~(uintptr_t)3);
    const uint32_t sh = (uint32_t)(a & 3);
    uint32_t v[9];
#pragma unroll
    for (int i = 0; i < 9; i++) v[i] = w[i];
#pragma unroll
    for (int i = 0; i < kPreW; i++) {
      const uint32_t lo = __builtin_amdgcn_alignbyte(v[2 * i + 1], v[2 * i], sh);
      const uint32_t hi = __builtin_amdgcn_alignbyte(v[2 * i + 2], v[2 * i + 1], sh);
      o[i] = ((uint64_t)hi << 32) | lo;
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < kPreW; i++) o[i] = 0;
  for (uint32_t i = 0; i < avail && i < 8 * kPreW; i++) o[i >> 3] |= (uint64_t)p[i] << (8 * (i & 7));
}

// kHist: streaming chunks with a history table; kParts: some stream carries a part index
// (lagging external sources) -- separate builds of the walk
template <int kTile, bool kHist, bool kParts>
__global__ __launch_bounds__(kTile) void find_matches_kernel(const Job *jobs, const uint32_t *pos_job, const SegRef *seg_ref,
                                                             const uint32_t *sorted_keys, const uint32_t *sorted_vals,
                                                             uint32_t total, int depth, uint32_t max_dist, uint32_t *matches,
                                                             int flags) {
  __shared__ uint32_t skey[kTile + kBack];
  __shared__ uint32_t spos[kTile + kBack];
  __shared__ uint64_t spre[kPreW][kTile + kBack];
  // xcd_order (an experiment, off): blocks are dealt round-robin over the 8 XCDs (b and b + 8
  // share one, MI355X_MICROARCH.md), so block b takes tile (b % 8) * per + b / 8 -- each XCD
  // sweeps one contiguous eighth of the sorted entries, a few streams at a time, meant to keep
  // the prefixes its tiles gather in its 4 MiB L2 (measured: no faster)
  // flags (experiments): 1 the XCD order; 8 records stored in SORTED order (wrong streams:
  // for timing the kernel without its scattered stores only)
  const int xcd_order = flags & 1;
  const bool sorted_store = flags & 8;
  const uint32_t ntiles = (total + kTile - 1) / kTile, per = (ntiles + 7) / 8;
  const uint32_t tix = xcd_order ? (blockIdx.x & 7) * per + (blockIdx.x >> 3) : blockIdx.x;
  if (tix >= ntiles) return;
  const uint32_t r0 = tix * kTile;
  // Each stream's positions are sorted within the stream's own range of global positions
  // (enc_sort.hip), so the tile's entries -- 256 within one 64 KiB range -- are all of one
  // stream: one SegRef for the block instead of a dependent lookup per entry.  Lookback
  // entries of the stream before are never candidates (the walk stops at them): no prefix.
  const SegRef sr = seg_ref[r0 >> kSegBits];
  for (int t = threadIdx.x; t < kTile + kBack; t += kTile) {
    int64_t r = (int64_t)r0 - kBack + t;
    uint32_t key = 0xFFFFFFFEu, g = 0;
    uint64_t pre[kPreW] = {0, 0, 0, 0};
    if (r >= 0 && r < (int64_t)total) {
      key = sorted_keys[r];
      g = sorted_vals[r];
      if ((key & kInvalidKey) == 0 && g >= sr.pos_base) load_prefix32(sr.base + g, sr.end - g, pre);
    }
    skey[t] = key;
    spos[t] = g;
#pragma unroll
    for (int i = 0; i < kPreW; i++) spre[i][t] = pre[i];
  }
  __syncthreads();
  // Each entry's candidates are the entries before it in its bucket run (same key, same
  // stream): the run's first index by a segmented max-scan -- a flag where the key or the
  // stream changes, the wave's prefix maximum of the flagged indices, the chunks before it
  // carried through LDS -- so the walk's trip count is known and its loop reads no keys.
  // (Wave w scans entries kBack + 64 w .. + 63; wave 0 also the kBack lookback entries.)
  __shared__ int chunk_last[kTile / 64 + 1];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  auto run_flag = [&](int e) -> int {   // e > 0
    return (skey[e] != skey[e - 1] || spos[e - 1] < sr.pos_base) ? e : -1;
  };
  auto wave_max_scan = [&](int v) -> int {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int u = __shfl_up(v, o);
      v = lane >= o ? max(v, u) : v;
    }
    return v;
  };
  const int me = kBack + threadIdx.x;
  int st_local = wave_max_scan(run_flag(me));
  if (lane == 63) chunk_last[wv + 1] = st_local;
  if (wv == 0) {
    const int lb = wave_max_scan(lane == 0 ? 0 : run_flag(lane));
    if (lane == 63) chunk_last[0] = lb;   // (>= 0: entry 0 starts a run)
  }
  __syncthreads();
  if (st_local < 0) {
    int c = chunk_last[0];
    for (int q = 1; q <= wv; q++) c = max(c, chunk_last[q]);
    st_local = c;
  }
  const int nrun = me - st_local;   // the entries before me in my run
  const uint32_t r = r0 + threadIdx.x;
  if (r >= total) return;
  const uint32_t key = skey[me], g = spos[me];
  int cnt = 0;
  if ((key & kInvalidKey) == 0) {
    const uint32_t p = g - sr.pos_base;
    // (pos_base is a multiple of the segment: the segment's end in global positions)
    const uint32_t limit = min(((g >> kSegBits) + 1) << kSegBits, sr.end) - g;   // copies never cross a parse segment
    const uint8_t *cur = sr.base + g;
    const Job &jb = jobs[(kHist || kParts) ? pos_job[r0 >> kSegBits] : 0];   // (the streaming / part-index fields)
    const bool parts = kParts && jb.parts;
    const uint32_t pA = (kHist || kParts) ? jb.abs_base + p : 0u, pbits = kParts ? jb.part_bits : 16u,
                   plag = kParts ? jb.part_lag : 0u;
    uint32_t best = 3;
    uint32_t local[kMaxMatches] = {};
    if constexpr (!kHist) {
      const uint64_t mine0 = spre[0][me];
      const int dmax = min(depth, kBack), nwalk = min(dmax, nrun);
      // The walk steps t in lockstep over the wave (a scalar loop: the run's end per lane is a
      // compare, not a divergent exit) and screens each candidate by its first word: it needs the
      // exact tests below iff the word's low best + 1 bytes all match (first difference past byte
      // best, or none in the word) or it lies beyond the window.  Most candidates fail the screen,
      // ~25 instructions each; the exact tests run under a branch the wave skips when no lane
      // needs them.  (As one per-lane loop with break / continue every candidate paid the exit-mask
      // bookkeeping of the rare paths, ~48 instructions, r05 ISA listing; as a per-lane skip loop
      // the lanes' different skip lengths multiplied the steps.)  Same candidates, same order,
      // same records.
      auto low_bytes = [](uint32_t n) -> uint64_t { return n >= 7 ? ~0ull : (1ull << (8 * (n + 1))) - 1; };
      uint64_t bmask = low_bytes(best);
      int tend = best >= limit ? 0 : nwalk;   // this lane's last step (0: done)
      // The walk ends before the first candidate beyond the window (positions ascend in a run,
      // so distances grow with t): found up front -- by a binary search in the rare run that
      // reaches that far -- so the steps need no distance, and read only the candidate's word.
      if (tend > 0 && g - spos[me - nwalk] > max_dist) {
        int lo = 0, hi = nwalk;   // d(lo) <= max_dist < d(hi)
        while (hi - lo > 1) {
          const int mid = (lo + hi) >> 1;
          if (g - spos[me - mid] > max_dist) hi = mid;
          else lo = mid;
        }
        tend = lo;
      }
      for (int t = 1; t <= kBack; t++) {
        if (__ballot(t <= tend) == 0) break;
        const int e = me - t;   // (>= 0: me >= kBack; lanes past their run read another run's entry, unused)
        const uint64_t x0 = mine0 ^ spre[0][e];
        if (!((t <= tend) & ((x0 & bmask) == 0))) continue;
        const uint32_t d = g - spos[e];
        const uint32_t qlen = (uint32_t)(__ffsll((unsigned long long)x0) - 1) >> 3;   // (x0 == 0: not used)
        const uint32_t pc = parts ? part_cap(pA, d, pbits, plag) : ~0u;   // part index: lagging source
        if (pc <= best) continue;
        uint32_t len;
        if (x0) {
          len = qlen;
        } else {
          // a candidate can only beat `best` if it matches byte `best` too
          if (best < 8 * kPreW) {
            const uint32_t sh = 8 * (best & 7);
            if (((spre[best >> 3][me] ^ spre[best >> 3][e]) >> sh) & 0xFF) continue;
          } else if (cur[best] != (cur - d)[best]) {
            continue;
          }
          len = 8 * kPreW;
#pragma unroll
          for (int w = 1; w < kPreW; w++) {
            const uint64_t x = spre[w][me] ^ spre[w][e];
            if (x) {
              len = 8 * w + ((uint32_t)(__ffsll((unsigned long long)x) - 1) >> 3);
              break;
            }
          }
          if (len == 8 * kPreW) {
            // measured up to the saturation length: the parse measures longer copies itself
            const uint32_t lim = min(limit, kMatchLenSat);
            if (lim > len) len += match_len(cur + len, (cur - d) + len, lim - len);
          }
        }
        len = min(min(len, limit), pc);
        if (len > best) {
          best = len;
          if (cnt == kMaxMatches) {   // keep the longest ones: drop the shortest
            for (int q = 1; q < kMaxMatches; q++) local[q - 1] = local[q];
            cnt--;
          }
          local[cnt++] = pack_match(d, len);
          bmask = low_bytes(best);
          // the parse measures a long copy itself; best >= limit ends the walk as well
          if (len >= limit || len >= kMatchLenSat) tend = 0;
        }
      }
      } else {
      const uint64_t mine0 = spre[0][me];
      // a candidate at distance d measured to len: the staircase keeps strictly longer ones;
      // DONE: no longer candidate can matter (the parse measures a long copy itself)
#define TAKE(d_, len_, DONE)                                               \
    do {                                                                     \
      const uint32_t l_ = min(min((len_), limit),                            \
                              parts ? part_cap(pA, (d_), pbits, plag) : ~0u);   \
      if (l_ > best) {                                                       \
        best = l_;                                                           \
        if (cnt == kMaxMatches) {                                            \
          for (int q = 1; q < kMaxMatches; q++) local[q - 1] = local[q];     \
          cnt--;                                                             \
        }                                                                    \
        local[cnt++] = pack_match((d_), l_);                                 \
        if (l_ >= limit || l_ >= kMatchLenSat) DONE;                         \
      }                                                                      \
    } while (0)
      const int dmax = min(depth, kBack);
      const int nwalk = min(dmax, nrun);
      // (the window walk as in the window-only build above: lockstep steps, the first word's
      // screen, the window end found up front; `stop` skips the history part as the serial walk's
      // break did -- at a candidate beyond the window, or once a copy reaches the limit)
      auto low_bytes = [](uint32_t n) -> uint64_t { return n >= 7 ? ~0ull : (1ull << (8 * (n + 1))) - 1; };
      uint64_t bmask = low_bytes(best);
      bool stop = nwalk > 0 && best >= limit;
      int tend = stop ? 0 : nwalk;
      if (tend > 0 && g - spos[me - nwalk] > max_dist) {
        int lo = 0, hi = nwalk;   // d(lo) <= max_dist < d(hi)
        while (hi - lo > 1) {
          const int mid = (lo + hi) >> 1;
          if (g - spos[me - mid] > max_dist) hi = mid;
          else lo = mid;
        }
        tend = lo;
        stop = true;
      }
      for (int s = 1; s <= kBack; s++) {
        if (__ballot(s <= tend) == 0) break;
        const int e = me - s;
        const uint64_t x0 = mine0 ^ spre[0][e];
        if (!((s <= tend) & ((x0 & bmask) == 0))) continue;
        const uint32_t d = g - spos[e];
        const uint32_t qlen = (uint32_t)(__ffsll((unsigned long long)x0) - 1) >> 3;   // (x0 == 0: not used)
        uint32_t len;
        if (x0) {
          len = qlen;
        } else {
          // a candidate can only beat `best` if it matches byte `best` too
          if (best < 8 * kPreW) {
            const uint32_t sh = 8 * (best & 7);
            if (((spre[best >> 3][me] ^ spre[best >> 3][e]) >> sh) & 0xFF) continue;
          } else if (cur[best] != (cur - d)[best]) {
            continue;
          }
          len = 8 * kPreW;
#pragma unroll
          for (int w = 1; w < kPreW; w++) {
            const uint64_t x = spre[w][me] ^ spre[w][e];
            if (x) {
              len = 8 * w + ((uint32_t)(__ffsll((unsigned long long)x) - 1) >> 3);
              break;
            }
          }
          if (len == 8 * kPreW) {
            // measured up to the saturation length: the parse measures longer copies itself
            const uint32_t lim = min(limit, kMatchLenSat);
            if (lim > len) len += match_len(cur + len, (cur - d) + len, lim - len);
          }
        }
        bool fin = false;
        TAKE(d, len, fin = true);
        bmask = low_bytes(best);
        if (fin) {
          stop = true;
          tend = 0;
        }
      }
      int t = nwalk + 1;   // (the history part's candidates count on from the window's)
      // streaming: then the bucket's occurrences before this chunk (farther, newest first)
      if (kHist && jb.hist_tab && !stop && t <= dmax) {
        const uint32_t *slot = jb.hist_tab + (size_t)(key & ((1u << kHashBits) - 1)) * kHistWays;
        const uint32_t A = jb.abs_base + p;
        const uint32_t reach = min(max_dist, p + jb.hist);
        for (int k = 0; k < kHistWays && t <= dmax && best < limit; k++, t++) {
          const uint32_t c = slot[k];
          if (c == kNoPos) break;
          const uint32_t d = A - c;
          if (d == 0 || d > reach) break;
          const uint8_t *cand = cur - d;
          if (cur[best] != cand[best]) continue;
          const uint32_t lim = min(limit, kMatchLenSat);
          bool fin = false;
          TAKE(d, match_len(cur, cand, lim), fin = true);
          if (fin) break;
        }
      }
#undef TAKE
    }
    // a match word is never 0 (length >= 4): the unused tail entries mark the count
    rec_store(matches + (uint64_t)(sorted_store ? r : g) * kMatchRec, local);
    return;
  }
  const uint32_t none[kMaxMatches] = {};
  rec_store(matches + (uint64_t)(sorted_store ? r : g) * kMatchRec, none);   // no candidates
}

// ---------------------------------------------------------------- near matches (short scan)
// findAllMatches' first step (hash-binary-tree.ts:167-194): before the tree, the positions up
// to kNear back are scanned nearest first for a copy of at least 2 bytes, until one of at least
// 3 is found -- the short, cheap-distance copies the bucket keys (6 bytes in GENERIC / TEXT
// mode, 4 in FONT mode) never offer.  Block = 256 consecutive positions of one stream (one
// segment): the 2-byte words of the block and the kNear positions before it are staged in LDS
// (one aligned b32 read per candidate), the bytes after each position for measuring.  The
// entries found are merged into the position's staircase record in front of the tree matches
// they dominate (every tree match at least as short; a nearer one would have been found first);
// a full record keeps its longest entries, as find_matches does.
constexpr int kNear = 64;        // the reference's shortMatchMaxBackward at q11
constexpr int kNearMeasure = 32; // near copies are measured up to this length (longer: the tree's)
constexpr int kNearT = 256;      // threads per block; a tile is kNearT - 1 positions (+ one for m3)
constexpr int kNearSpan = 4096;  // positions per block (its fixed lookups amortised)
template <bool kHist, bool kParts>
__global__ __launch_bounds__(kNearT) void near_matches_kernel(const Job *jobs, const uint32_t *pos_job, const SegRef *seg_ref,
                                                              uint32_t total, uint32_t max_dist, uint32_t *matches) {
  constexpr int kW = kNear + kNearT + kNearMeasure;   // staged words per tile
  constexpr int kPer = (kW + kNearT - 1) / kNearT;    // ... per thread
  constexpr uint32_t kStep = kNearT - 1;
  __shared__ uint32_t w4[kPer * kNearT];    // the 4 bytes at each staged offset (zero outside the stream)
  __shared__ uint32_t sm2[2][kNearT];       // each position's 2-byte candidate mask (lo, hi word)
  const uint32_t gb = blockIdx.x * kNearSpan;   // (a block stays inside one 64 KiB segment)
  if (gb >= total) return;
  const SegRef sr = seg_ref[gb >> kSegBits];
  if (gb >= sr.end) return;   // padding, or an uncompressed stream's positions
  const Job &jb = jobs[pos_job[gb >> kSegBits]];
  const uint32_t hist = kHist ? jb.hist : 0u;   // bytes before data[0] copies may reach (streaming)
  const uint32_t n = sr.end - sr.pos_base;
  const uint32_t pbits = kParts ? jb.part_bits : 16u, plag = kParts ? jb.part_lag : 0u;
  const bool parts = kParts && jb.parts;
  const uint32_t t = threadIdx.x;
  typedef const __attribute__((address_space(1))) uint32_t GU32;
  // the tile's words, loaded one tile ahead (kPer per thread, in registers): word i = the 4
  // bytes at g0 - kNear + i, each 0 outside [the earliest reachable byte, the stream's end).
  // Inside, from two aligned dwords; at the edges byte by byte.
  uint32_t nw[kPer];
  auto load_tile = [&](uint32_t g0) {
    const int64_t p0 = (int64_t)g0 - sr.pos_base;
    const int64_t lo = -(int64_t)min((uint64_t)p0 + hist, (uint64_t)kNear);   // earliest offset with a byte
#pragma unroll
    for (int k = 0; k < kPer; k++) {
      const int i = k * kNearT + (int)t;
      const int64_t o = (int64_t)i - kNear, q = p0 + o;   // the word's first byte, stream-relative
      uint32_t v = 0;
      if (i < kW && g0 < sr.end) {
        if (o >= lo && q + 8 <= (int64_t)n) {
          const uintptr_t a = (uintptr_t)(sr.base + (int64_t)g0 + o);
          GU32 *w = (GU32 *)(a & ~(uintptr_t)3);
          v = __builtin_amdgcn_alignbyte(w[1], w[0], (uint32_t)(a & 3));
        } else {
#pragma unroll
          for (int b = 0; b < 4; b++)
            if (o + b >= lo && q + b < (int64_t)n) v |= (uint32_t)sr.base[(int64_t)g0 + o + b] << (8 * b);
        }
      }
      nw[k] = v;
    }
  };
  load_tile(gb);
  for (uint32_t g0 = gb; g0 < gb + kNearSpan && g0 < sr.end; g0 += kStep) {
    __syncthreads();   // (the previous tile's readers are done)
#pragma unroll
    for (int k = 0; k < kPer; k++) w4[k * kNearT + t] = nw[k];
    load_tile(g0 + kStep);   // in flight during this tile
    __syncthreads();
    const uint32_t x = kNear + t, g = g0 + t, p = g - sr.pos_base;
    const bool here = g < sr.end && p + 2 <= n;
    // bit d of m2: the byte pair at p matches the pair d back (1 <= d <= reach).  One LDS word
    // holds two candidate pairs (its low half the pair at y, its high half the pair at y + 2),
    // tested at once: 32 words for the 63 distances, a zero-half test per word.
    const uint32_t reach = min(min((uint32_t)kNear - 1, max_dist), p + hist);   // (the reference's d < 64)
    const uint32_t me = w4[x] & 0xFFFFu, pp = me | (me << 16);
    // Per word a packed 16-bit min with 1 gives each half's "differs" bit (v_pk_min_u16: bit 0
    // for the low half, bit 16 for the high); two words' bits are gathered two at a time into
    // acc (bits 2k, 2k + 1: the low halves, d = 4k + 2, 4k + 3; bits 16 + 2k, 17 + 2k: the high
    // halves, d = 4k, 4k + 1), ~6 VALU ops a k where the zero-half tests and the nibble took
    // ~20; the bits are put in distance order once at the end.
    // (asm: written as a vector min, the compiler turned it into two compares and selects a half)
    auto differs = [](uint32_t v) -> uint32_t {
      uint32_t r;
      asm("v_pk_min_u16 %0, %1, %2" : "=v"(r) : "v"(v), "s"(0x00010001u));
      return r;
    };
    uint32_t acc[2] = {0u, 0u};
#pragma unroll
    for (int k = 0; k < 16; k++) {
      // y = x - 4k - 2: pairs at d = 4k + 2 (low half), 4k (high); y = x - 4k - 3: 4k + 3, 4k + 1
      const uint32_t ve = w4[x - 4 * k - 2] ^ pp, vo = w4[x - 4 * k - 3] ^ pp;
      acc[k >> 3] |= (differs(ve) | (differs(vo) << 1)) << (2 * (k & 7));
    }
    // (the 2-bit groups of a 16-bit half spread to every other 2-bit slot)
    auto spread2 = [](uint32_t v) -> uint32_t {
      v = (v | (v << 8)) & 0x00FF00FFu;
      v = (v | (v << 4)) & 0x0F0F0F0Fu;
      return (v | (v << 2)) & 0x33333333u;
    };
    const uint32_t ea = ~acc[0], eb = ~acc[1];   // 1: the pair matches
    const uint32_t ml = spread2(ea >> 16) | (spread2(ea & 0xFFFFu) << 2);
    const uint32_t mh = spread2(eb >> 16) | (spread2(eb & 0xFFFFu) << 2);
    const uint64_t valid = reach >= 63 ? ~1ull : ((2ull << reach) - 2ull);   // bits 1 .. reach
    const uint64_t m2 = here ? ((((uint64_t)mh << 32) | ml) & valid) : 0ull;
    sm2[0][t] = (uint32_t)m2;
    sm2[1][t] = (uint32_t)(m2 >> 32);
    // the position's record, loaded before the exchange so the barrier hides its latency
    uint32_t *rec = matches + (uint64_t)g * kMatchRec;
    // (thread kStep, and a position past the block: the m2 of the position before it only)
    const bool emit = here && m2 && t < kStep && g < gb + kNearSpan;
    uint32_t old[kMaxMatches] = {};
    if (emit) rec_load(rec, old);
    __syncthreads();
    if (!emit) continue;
    // a 3-byte copy from d = the pairs at p and at p + 1 both match d back
    const uint64_t m3 = m2 & (((uint64_t)sm2[1][t + 1] << 32) | sm2[0][t + 1]);
    const uint32_t limit = min(((g >> kSegBits) + 1) << kSegBits, sr.end) - g;   // copies never cross a parse segment
    const uint32_t pA = kParts ? jb.abs_base + p : 0u;
    const uint32_t cap0 = min(limit, (uint32_t)kNearMeasure);
    // the reference's scan (nearest first, until a copy of 3 bytes or more) keeps the nearest
    // 2-byte copy if it is nearer than the nearest 3-byte one, and that one, measured
    uint32_t f0 = 0, f1 = 0, best = 1;
    const uint32_t d2 = (uint32_t)__ffsll((unsigned long long)m2) - 1u;
    const uint32_t d3 = m3 ? (uint32_t)__ffsll((unsigned long long)m3) - 1u : 64u;
    if (d2 < d3) {   // a 2-byte copy nearer than any longer one
      const uint32_t cap = min(cap0, parts ? part_cap(pA, d2, pbits, plag) : ~0u);
      if (cap >= 2) {
        f0 = pack_match(d2, 2);
        best = 2;
      }
    }
    if (d3 < 64u) {
      const uint32_t cap = min(cap0, parts ? part_cap(pA, d3, pbits, plag) : ~0u);
      // measured a word at a time (up to kNearMeasure)
      uint32_t len = kNearMeasure;
      for (int k = 0; k < kNearMeasure / 4; k++) {
        const uint32_t v = w4[x + 4 * k] ^ w4[x - d3 + 4 * k];
        if (v) {
          len = 4 * k + ((uint32_t)(__ffs(v) - 1) >> 3);
          break;
        }
      }
      len = min(len, cap);
      if (len > best) {
        best = len;
        if (f0) f1 = pack_match(d3, len);
        else f0 = pack_match(d3, len);
      }
    }
    if (!f0) continue;
    if (old[0] && (match_dist(old[0]) == kCDictMark || (jb.dict && is_dict(match_dist(old[0]))))) continue;   // a dictionary copy: the only entry
    // the near entries, then the tree's longer ones; a full record keeps its longest
    uint32_t w[2 + kMaxMatches];
    int m = 0;
    w[m++] = f0;
    if (f1) w[m++] = f1;
#pragma unroll
    for (int q = 0; q < kMaxMatches; q++)
      if (old[q] && match_length(old[q]) > best) w[m++] = old[q];
    const int sk = m > kMaxMatches ? m - kMaxMatches : 0;
    uint32_t o4[kMaxMatches] = {};
#pragma unroll
    for (int q = 0; q < kMaxMatches; q++)
      if (q + sk < m) o4[q] = w[q + sk];
    rec_store(rec, o4);
  }
}

void launch_near_matches(hipStream_t st, const Job *jobs, const uint32_t *pos_job, const SegRef *seg_ref, uint32_t total,
                         uint32_t max_dist, bool hist, bool parts, uint32_t *matches) {
  const dim3 g((total + kNearSpan - 1) / kNearSpan), b(kNearT);
  if (hist && parts) hipLaunchKernelGGL((near_matches_kernel<true, true>), g, b, 0, st, jobs, pos_job, seg_ref, total, max_dist, matches);
  else if (hist) hipLaunchKernelGGL((near_matches_kernel<true, false>), g, b, 0, st, jobs, pos_job, seg_ref, total, max_dist, matches);
  else if (parts) hipLaunchKernelGGL((near_matches_kernel<false, true>), g, b, 0, st, jobs, pos_job, seg_ref, total, max_dist, matches);
  else hipLaunchKernelGGL((near_matches_kernel<false, false>), g, b, 0, st, jobs, pos_job, seg_ref, total, max_dist, matches);
}

// ---------------------------------------------------------------- streaming history update
// After a chunk's matches: every bucket the chunk touched gets its newest kHistWays stream
// positions (this chunk's, from the end of its sorted run, then the older table entries).
// The thread at a run's end owns the bucket: no two threads write one slot.
__global__ void hist_update_kernel(const Job *jobs, const uint32_t *pos_job, const uint32_t *sorted_keys,
                                   const uint32_t *sorted_vals, uint32_t total) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= total) return;
  const uint32_t key = sorted_keys[r];
  if (key & kInvalidKey) return;
  const uint32_t g = sorted_vals[r];
  const uint32_t j = pos_job[g >> kSegBits];
  const Job &jb = jobs[j];
  if (!jb.hist_tab) return;
  if (r + 1 < total && sorted_keys[r + 1] == key && pos_job[sorted_vals[r + 1] >> kSegBits] == j) return;   // not the run's end
  uint32_t *slot = jb.hist_tab + (size_t)(key & ((1u << kHashBits) - 1)) * kHistWays;
  uint32_t nw[kHistWays];
  int m = 0;
  for (uint32_t q = r; m < kHistWays; q--) {
    const uint32_t gq = sorted_vals[q];
    nw[m++] = jb.abs_base + (gq - jb.pos_base);
    if (q == 0 || sorted_keys[q - 1] != key || sorted_vals[q - 1] < jb.pos_base) break;
  }
  uint32_t old[kHistWays];
  for (int k = 0; k < kHistWays; k++) old[k] = slot[k];
  for (int k = m; k < kHistWays; k++) nw[k] = old[k - m];
  for (int k = 0; k < kHistWays; k++) slot[k] = nw[k];
}

// ---------------------------------------------------------------- literal cost model per stream
__global__ void lit_histo_kernel(const Job *jobs, const Seg *segs, uint32_t *lit_histo /*256 per job*/) {
  __shared__ uint32_t h[256];
  const Seg sg = segs[blockIdx.x];
  const Job &jb = jobs[sg.job];
  for (int i = threadIdx.x; i < 256; i += blockDim.x) h[i] = 0;
  __syncthreads();
  for (uint32_t p = sg.start + threadIdx.x; p < sg.end; p += blockDim.x) atomicAdd(&h[jb.data[p]], 1u);
  __syncthreads();
  for (int i = threadIdx.x; i < 256; i += blockDim.x)
    if (h[i]) atomicAdd(&lit_histo[sg.job * 256 + i], h[i]);
}


// ---------------------------------------------------------------- static-dictionary words
// After the window walk, over the first dict_span bytes of every stream (where the window is
// short): a position with no window match gets the longest RFC 7932 word (identity
// transform) of its bucket that the input repeats in full -- a word reference cannot be cut,
// and it may not cross the parse segment.  Block = 256 consecutive positions of one stream.
__global__ __launch_bounds__(256) void dict_matches_kernel(const Job *jobs, int njobs, const uint32_t *dict_tab,
                                                           const uint8_t *dict_data, uint32_t *matches) {
  for (int j = blockIdx.y; j < njobs; j += gridDim.y) {
  const Job &jb = jobs[j];
  const uint32_t p = blockIdx.x * 256 + threadIdx.x;
  if (!jb.dict || p >= min(jb.dict_span, jb.n) || p + 4 > jb.n) continue;
  uint32_t *rec = matches + (uint64_t)(jb.pos_base + p) * kMatchRec;
  if (rec[0] != 0) continue;   // the window has a match here
  const uint32_t limit = min(((p >> kSegBits) + 1) << kSegBits, jb.n) - p;
  const uint8_t *cur = jb.data + p;
  const uint32_t *slot = dict_tab + (size_t)dict_hash(load_u32(cur)) * kDictWays;
  for (int k = 0; k < kDictWays; k++) {
    const uint32_t e = slot[k];
    if (!e) break;
    const uint32_t L = e >> 16, idx = e & 0x7FF;
    if (L > limit) continue;
    // dict_data: the word-list offsets per length (32 x u32), then the RFC 7932 words
    const uint8_t *w = dict_data + 128 + reinterpret_cast<const uint32_t *>(dict_data)[L] + idx * L;
    uint32_t i = 0;
    while (i < L && w[i] == cur[i]) i++;
    if (i == L) {
      rec[0] = pack_match(kDictFlag | idx, L);
      break;
    }
  }
  }
}

// ---------------------------------------------------------------- custom-dictionary copies
// (kCDictMark, enc_common.h.)  Thread per stream position q: where the four bytes ending at q
// equal the dictionary's last four, the common suffix of the input up to q and of the
// dictionary is measured backwards (within q's parse segment, at most kLongCopy bytes); the
// copy of that length starting at p = q - L + 1 is offered at p if the window found nothing
// there.  Several q may offer one p: the longest wins (a compare-and-swap maximum, so the
// result does not depend on thread order).
__global__ __launch_bounds__(256) void cdict_matches_kernel(const Job *jobs, const uint32_t *pos_job, uint32_t total,
                                                            uint32_t *matches) {
  for (uint32_t g = blockIdx.x * 256 + threadIdx.x; g < total; g += gridDim.x * 256) {
    const Job &jb = jobs[pos_job[g >> kSegBits]];
    if (!jb.cdict) continue;
    const uint32_t q = g - jb.pos_base;
    if (q < 3 || q >= jb.n) continue;
    const uint8_t *d = jb.data;
    if (load_u32(d + q - 3) != jb.cdict_tail4) continue;
    const uint32_t seg0 = (q >> kSegBits) << kSegBits;
    const uint32_t cap = min(min((uint32_t)kLongCopy, jb.cdict_len), q - seg0 + 1);
    const uint8_t *t = jb.cdict + jb.cdict_len;   // one past the dictionary's last byte
    uint32_t L = 4;
    while (L < cap && d[q - L] == t[-1 - (int)L]) L++;
    if (L > cap) continue;   // (a dictionary or segment of fewer than four bytes)
    uint32_t *rec = matches + (uint64_t)(g - L + 1) * kMatchRec;
    const uint32_t mine = pack_match(kCDictMark, L);
    uint32_t old = rec[0];
    while ((old == 0u || match_dist(old) == kCDictMark) && old < mine) {
      const uint32_t prev = atomicCAS(rec, old, mine);
      if (prev == old) break;
      old = prev;
    }
  }
}
void launch_cdict_matches(hipStream_t st, const Job *jobs, const uint32_t *pos_job, uint32_t total, uint32_t *matches) {
  const unsigned grid = (unsigned)std::min<uint64_t>(16384, (total + 255) / 256);
  hipLaunchKernelGGL(cdict_matches_kernel, dim3(grid), dim3(256), 0, st, jobs, pos_job, total, matches);
}

void launch_find_matches(hipStream_t st, const Job *jobs, const uint32_t *pos_job, const SegRef *seg_ref,
                         const uint32_t *skeys, const uint32_t *svals, uint32_t total, int depth, uint32_t max_dist,
                         bool hist, bool parts, uint32_t *matches) {
  // tile of sorted entries per block: each tile also stages the kBack entries before it
  // (MIB_FM_TILE: experiment knob, 256 / 512 / 1024)
  static const int tile = knob("MIB_FM_TILE") ? atoi(knob("MIB_FM_TILE")) : 256;
  // XCD-aware tile order (MIB_FM_XCD=1): measured no faster on C4 (64.9 vs 65.4 ms), off
  static const int xcd = knob("MIB_FM_XCD") ? atoi(knob("MIB_FM_XCD")) : 0;
  static const int flags = (xcd ? 1 : 0) | (knob("MIB_FM_SORTED_STORE") ? 8 : 0);
#define MIB_FM(T, H, P)                                                                                                   \
  hipLaunchKernelGGL((find_matches_kernel<T, H, P>), dim3(8 * (((total + T - 1) / T + 7) / 8)), dim3(T), 0, st, jobs, pos_job, \
                     seg_ref, skeys, svals, total, depth, max_dist, matches, flags)
#define MIB_FM_T(T)                            \
  do {                                         \
    if (hist && parts) MIB_FM(T, true, true);  \
    else if (hist) MIB_FM(T, true, false);     \
    else if (parts) MIB_FM(T, false, true);    \
    else MIB_FM(T, false, false);              \
  } while (0)
  if (tile >= 1024) MIB_FM_T(1024);
  else if (tile >= 512) MIB_FM_T(512);
  else MIB_FM_T(256);
#undef MIB_FM_T
#undef MIB_FM
}
void launch_hist_update(hipStream_t st, const Job *jobs, const uint32_t *pos_job, const uint32_t *skeys,
                        const uint32_t *svals, uint32_t total) {
  hipLaunchKernelGGL(hist_update_kernel, dim3((total + 255) / 256), dim3(256), 0, st, jobs, pos_job, skeys, svals, total);
}
void launch_dict_matches(hipStream_t st, const Job *jobs, int njobs, uint32_t span, const uint32_t *dict_tab,
                         const uint8_t *dict_data, uint32_t *matches) {
  if (!njobs || !span) return;
  hipLaunchKernelGGL(dict_matches_kernel, dim3((span + 255) / 256, std::min(njobs, 65535)), dim3(256), 0, st, jobs, njobs, dict_tab,
                     dict_data, matches);
}
void launch_lit_histo(hipStream_t st, const Job *jobs, const Seg *segs, int nsegs, uint32_t *lit_h) {
  hipLaunchKernelGGL(lit_histo_kernel, dim3(nsegs), dim3(256), 0, st, jobs, segs, lit_h);
}

}  // namespace enc
}  // namespace mib
