// brotli_amd: batch Brotli (RFC 7932) encoder for gfx950.
//
// The reference's quality-11 path (countertype/brotli-lib src/encode/encode.ts:181-281 ->
// createHqZopfliBackwardReferences backward-references-hq.ts:485-608 -> storeMetaBlock
// metablock.ts:504-761) is inherently serial per stream: an insertion-ordered binary tree
// (hash-binary-tree.ts:57-153) and a forward DP over every position.  This engine keeps the
// same algorithmic family -- hash-bucketed match finding, a cost-model shortest-path parse
// over (insert, copy, distance) commands, Huffman coding of literal / command / distance
// symbols -- but restructures each stage for a GPU:
//
//   1. hash_keys + radix sort: every position of every stream gets a 32-bit key
//      (job << 17 | hash4); a stable device radix sort groups each bucket with positions in
//      increasing order, i.e. every bucket is the reference's hash chain laid out flat.
//   2. find_matches: one lane per position walks its bucket backwards (the most recent
//      candidates first, depth by quality) and keeps the increasing-length / smallest-
//      distance staircase, as findAllMatches does (hash-binary-tree.ts:156-227).
//   3. dp: one wave per 64 KiB segment runs the shortest-path parse; the 64 lanes relax
//      the candidate copy lengths of a position in parallel (updateNodes,
//      backward-references-hq.ts:267-382, with one start candidate as at quality 10).
//   4. backtrack (lane per segment) -> assemble (lane per stream: distance cache and short
//      codes, command prefix codes, command.ts:83-179) -> histograms (atomics) ->
//      huffman (createHuffmanTree entropy-encode.ts:24-131 + tree serialisation
//      context-map.ts:215-347) -> sizes + scan -> emit (lane per segment, bit-exact
//      placement) -> pack.
//
// Segments are independent in the parse (a copy never crosses a segment end); the
// distance cache and insert lengths are stitched serially per stream in `assemble`, so the
// output is one valid RFC 7932 stream per input, decodable by any decoder.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "common.h"

extern "C" void mib_ctx_add_time(mib_ctx *c, const char *name, double ms);
extern "C" int mib_ctx_profiling(mib_ctx *c);
extern "C" void **mib_ctx_enc_ws(mib_ctx *c);

namespace mib {
namespace enc {

constexpr uint32_t kSegBits = 16;
constexpr uint32_t kSeg = 1u << kSegBits;     // 64 KiB parse segments
constexpr int kMaxMatches = 6;                // staircase entries kept per position
constexpr int kRing = 512;                    // DP node window (> kLongCopy + 64)
constexpr int kLongCopy = 325;                // MAX_ZOPFLI_LEN_QUALITY_11 (enc-constants.ts:33)
constexpr uint32_t kMaxMetablock = 1u << 24;  // encode.ts:206
constexpr uint32_t kInvalidKey = 0xFFFFFFFFu;

struct Job {                // one stream to encode
  const uint8_t *data;      // its bytes (device), readable up to n + 16
  uint32_t n;
  uint32_t pos_base;        // global position index of byte 0 (sort / per-position arrays)
  uint32_t seg_base;        // first segment
  uint32_t nseg;
  uint32_t mb_base;         // first metablock
  uint32_t nmb;
  uint32_t cmd_base;        // command array slice (capacity n/2 + nseg + 4)
  uint32_t ncmd;            // written by assemble
  uint32_t lgwin;
  uint32_t npostfix, ndirect;
  uint32_t uncompressed;    // 1: quality 0 / n < 64 path; 2: compressed form was larger
  uint32_t hdr_lgwin;       // window bits written before the first metablock, 0 = none
  uint32_t final_;          // last chunk of the stream: ISLAST metablock (else a byte-aligning flush)
  int32_t dc_in[4];         // distance cache at the start (streaming continues it)
  int32_t dc_out[4];        // and after the last command (written by assemble)
  uint64_t out_off;         // byte offset of its scratch output slice
  uint64_t out_cap;
  uint64_t total_bits;      // written by offsets / uncompressed
};

struct Seg {
  uint32_t job, start, end;   // stream-local [start, end)
  uint32_t mb;                // metablock index (global)
  uint32_t cmd_off;           // per-segment command scratch (capacity (end-start)/2 + 2)
  uint32_t ncmd;              // written by backtrack
  uint32_t tail_lits;         // literals after the last copy
  uint32_t pad;
  uint64_t bit_off;           // written by sizes
  uint64_t bits;
};

struct Mb {                   // one metablock
  uint32_t job, start, end;   // stream-local
  uint32_t first_seg, nseg;
  uint32_t cmd_first, ncmd;   // in the job's assembled command list
  uint32_t is_last;
  uint64_t hdr_bits;          // metablock header + trees (written by huffman)
  uint64_t bit_off;           // of the header, stream-relative
};

struct Cmd {                  // assembled command
  uint32_t ins, copy;         // copy == 0: trailing literal-only command
  uint32_t dist_extra;
  uint16_t cmd_prefix, dist_prefix;   // dist_prefix: code | nbits << 10 (command.ts:146-179)
};

struct RawCmd { uint32_t ins, len, dist; };

// ---------------------------------------------------------------- shared coding helpers (command.ts)
__device__ __forceinline__ int log2floor_u(uint32_t v) { return 31 - __clz(v); }
__device__ __constant__ uint32_t kInsBase[24] = {0, 1, 2, 3, 4, 5, 6, 8, 10, 14, 18, 26, 34, 50, 66, 98, 130, 194, 322, 578, 1090, 2114, 6210, 22594};
__device__ __constant__ uint32_t kInsExtra[24] = {0, 0, 0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 7, 8, 9, 10, 12, 14, 24};
__device__ __constant__ uint32_t kCopyBase[24] = {2, 3, 4, 5, 6, 7, 8, 9, 10, 12, 14, 18, 22, 30, 38, 54, 70, 102, 134, 198, 326, 582, 1094, 2118};
__device__ __constant__ uint32_t kCopyExtra[24] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 7, 8, 9, 10, 24};

__device__ __forceinline__ int ins_code(uint32_t n) {
  if (n < 6) return (int)n;
  if (n < 130) { int nb = log2floor_u(n - 2) - 1; return (nb << 1) + (int)((n - 2) >> nb) + 2; }
  if (n < 2114) return log2floor_u(n - 66) + 10;
  if (n < 6210) return 21;
  if (n < 22594) return 22;
  return 23;
}
__device__ __forceinline__ int copy_code(uint32_t n) {
  if (n < 10) return (int)n - 2;
  if (n < 134) { int nb = log2floor_u(n - 6) - 1; return (nb << 1) + (int)((n - 6) >> nb) + 4; }
  if (n < 2118) return log2floor_u(n - 70) + 12;
  return 23;
}
__device__ __forceinline__ int combine_codes(int ic, int cc, bool use_last) {
  int bits64 = (cc & 7) | ((ic & 7) << 3);
  if (use_last && ic < 8 && cc < 16) return cc < 8 ? bits64 : (bits64 | 64);
  int off = 2 * ((cc >> 3) + 3 * (ic >> 3));
  off = (off << 5) + 0x40 + ((0x520D40 >> off) & 0xC0);
  return off | bits64;
}
// prefixEncodeCopyDistance (command.ts:111-135): code | nbits << 10, extra
__device__ __forceinline__ uint32_t dist_prefix(uint32_t dcode, int ndirect, int npostfix, uint32_t *extra) {
  if (dcode < (uint32_t)(16 + ndirect)) {
    *extra = 0;
    return dcode;
  }
  uint32_t dist = (1u << (npostfix + 2)) + (dcode - 16 - (uint32_t)ndirect);
  int bucket = log2floor_u(dist) - 1;
  uint32_t pmask = (1u << npostfix) - 1, postfix = dist & pmask, prefix = (dist >> bucket) & 1;
  uint32_t offset = (2 + prefix) << bucket;
  uint32_t nbits = (uint32_t)(bucket - npostfix);
  *extra = (dist - offset) >> npostfix;
  return (nbits << 10) | (16 + (uint32_t)ndirect + ((2 * (nbits - 1) + prefix) << npostfix) + postfix);
}

__device__ __forceinline__ uint32_t load_u32(const uint8_t *p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
__device__ __forceinline__ uint32_t hash4(const uint8_t *p) { return (load_u32(p) * 0x1E35A7BDu) >> 15; }

// length of the common prefix of a[] and b[], up to limit
__device__ __forceinline__ uint32_t match_len(const uint8_t *a, const uint8_t *b, uint32_t limit) {
  uint32_t m = 0;
  while (m + 4 <= limit) {
    uint32_t x = load_u32(a + m) ^ load_u32(b + m);
    if (x) return m + (__ffs(x) - 1) / 8;
    m += 4;
  }
  while (m < limit && a[m] == b[m]) m++;
  return m;
}

// ---------------------------------------------------------------- 1. keys
// Every global position (including the padding after each stream) gets a key; padding and
// the last 3 bytes of a stream get the invalid key, which sorts after every real bucket.
__global__ void hash_keys_kernel(const Job *jobs, const uint32_t *pos_job, uint32_t total, uint32_t *keys, uint32_t *vals) {
  for (uint32_t g = blockIdx.x * blockDim.x + threadIdx.x; g < total; g += gridDim.x * blockDim.x) {
    uint32_t j = pos_job[g >> kSegBits];
    const Job &jb = jobs[j];
    uint32_t p = g - jb.pos_base;
    keys[g] = (p + 4 <= jb.n && !jb.uncompressed) ? ((j << 17) | hash4(jb.data + p)) : kInvalidKey;
    vals[g] = g;
  }
}
// ---------------------------------------------------------------- 2. matches
// One thread per SORTED entry: a bucket is a run of equal keys with positions ascending, so
// the candidates of entry r are entries r-1, r-2, ... (most recent first) -- the
// reference's hash chain / tree candidates (hash-binary-tree.ts:156-227), depth by
// quality.  A 256-entry tile plus the 64 entries before it is staged in LDS with the 8
// bytes following each position, so most candidates are rejected or measured without
// touching HBM; only matches of 8+ bytes extend through global memory.  The staircase of
// strictly increasing lengths (shortest distance for each length) is kept, longest last.
constexpr int kTile = 256;
constexpr int kBack = 64;

__device__ __forceinline__ uint64_t load_prefix8(const uint8_t *p, uint32_t avail) {
  if (avail >= 8) {
    uint64_t v = 0;
    for (int i = 0; i < 8; i++) v |= (uint64_t)p[i] << (8 * i);
    return v;
  }
  uint64_t v = 0;
  for (uint32_t i = 0; i < avail; i++) v |= (uint64_t)p[i] << (8 * i);
  return v;
}

__global__ __launch_bounds__(kTile) void find_matches_kernel(const Job *jobs, const uint32_t *sorted_keys,
                                                             const uint32_t *sorted_vals, uint32_t total, int depth,
                                                             uint64_t *matches, uint8_t *nmatch) {
  __shared__ uint32_t skey[kTile + kBack];
  __shared__ uint32_t spos[kTile + kBack];
  __shared__ uint64_t spre[kTile + kBack];
  const uint32_t r0 = blockIdx.x * kTile;
  for (int t = threadIdx.x; t < kTile + kBack; t += kTile) {
    int64_t r = (int64_t)r0 - kBack + t;
    uint32_t key = 0xFFFFFFFEu, g = 0;
    uint64_t pre = 0;
    if (r >= 0 && r < (int64_t)total) {
      key = sorted_keys[r];
      g = sorted_vals[r];
      if (key != kInvalidKey) {
        const Job &jb = jobs[key >> 17];
        uint32_t p = g - jb.pos_base;
        pre = load_prefix8(jb.data + p, jb.n - p);
      }
    }
    skey[t] = key;
    spos[t] = g;
    spre[t] = pre;
  }
  __syncthreads();
  const uint32_t r = r0 + threadIdx.x;
  if (r >= total) return;
  const int me = kBack + threadIdx.x;
  const uint32_t key = skey[me], g = spos[me];
  int cnt = 0;
  if (key != kInvalidKey) {
    const Job &jb = jobs[key >> 17];
    const uint32_t p = g - jb.pos_base;
    const uint32_t max_dist = (1u << jb.lgwin) - 16;
    const uint32_t seg_end = min(((p >> kSegBits) + 1) << kSegBits, jb.n);
    const uint32_t limit = seg_end - p;   // copies never cross a parse segment
    const uint8_t *cur = jb.data + p;
    const uint64_t mine = spre[me];
    uint32_t best = 3;
    uint64_t local[kMaxMatches];
    const int dmax = min(depth, kBack);
    for (int t = 1; t <= dmax; t++) {
      const int e = me - t;
      if (skey[e] != key) break;
      const uint32_t d = g - spos[e];
      if (d > max_dist || best >= limit) break;
      const uint64_t x = mine ^ spre[e];
      uint32_t len;
      if (x) {
        len = (uint32_t)(__ffsll((unsigned long long)x) - 1) >> 3;
        if (len <= best) continue;
        len = min(len, limit);
      } else {
        const uint8_t *cand = cur - d;
        if (best >= 8 && cur[best] != cand[best]) continue;
        len = 8 + match_len(cur + 8, cand + 8, limit > 8 ? limit - 8 : 0);
        len = min(len, limit);
      }
      len = min(len, 65535u);   // copy lengths travel as u16 through the parse
      if (len > best) {
        best = len;
        if (cnt == kMaxMatches) {   // keep the longest ones: drop the shortest
          for (int q = 1; q < kMaxMatches; q++) local[q - 1] = local[q];
          cnt--;
        }
        local[cnt++] = ((uint64_t)d << 32) | len;
        if (len >= limit || len >= 4096) break;
      }
    }
    for (int q = 0; q < cnt; q++) matches[(uint64_t)g * kMaxMatches + q] = local[q];
  }
  nmatch[g] = (uint8_t)cnt;
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
// The DP block is one wave: LDS traffic of a wave is processed in order, so a compiler
// fence at wavefront scope is all the lanes need between dependent LDS steps (a
// workgroup barrier would also drain the outstanding global stores/loads every time).
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}
constexpr int kWin = kBatch + 64;
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
  __shared__ float litc[256];
  __shared__ float cmdc[704];
  __shared__ float distc[128];
  __shared__ uint8_t win[kWin];
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
  wave_sync();
  const uint32_t a = sg.start, b = sg.end;
  const uint32_t gbase = jb.pos_base;
  if (lane == 0) cost[a % kRing] = 0.f;
  // the path's last distance: verified run [c_from, c_upto) of data[p] == data[p - c_ld]
  uint32_t c_ld = 0, c_from = 0, c_upto = 0;
  bool c_end = false;   // c_upto is a mismatch (or the segment end), not just "verified so far"
  uint32_t i = a;
  while (i < b) {
    // ---- stage the next batch: matches and their distance costs, literal bytes
    const uint32_t i0 = i;
    const uint32_t nb = min((uint32_t)kBatch, b - i0);
    wave_sync();
    {
      int nm = 0;
      if ((uint32_t)lane < nb) nm = nmatch[gbase + i0 + lane];
      bnm[lane] = (uint8_t)nm;
      const uint64_t *src = matches + (uint64_t)(gbase + i0 + lane) * kMaxMatches;
      for (int q = 0; q < nm; q++) {
        uint64_t m = src[q];
        uint32_t extra;
        uint32_t dp = dist_prefix((uint32_t)(m >> 32) + 15, (int)jb.ndirect, (int)jb.npostfix, &extra);
        bmt[lane * kMaxMatches + q] = m;
        bmc[lane * kMaxMatches + q] = (float)(dp >> 10) + distc[min(dp & 0x3FFu, 127u)];
      }
      for (int t = lane; t < kWin; t += 64) win[t] = (i0 + t < b) ? data[i0 + t] : 0;
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
      wave_sync();
      if (lane == 0) {
        cost[slot] = kInf;   // the slot now serves position i + kRing
        const int ns = (i + 1) % kRing;
        const float c = ci + litc[win[off]];
        if (c < cost[ns]) {
          cost[ns] = c;
          meta[ns] = pack_node(ld, 0, ins_i + 1);
        }
      }
      wave_sync();
      const int ic = ins_code(ins_i);
      const float base = ci + (float)kInsExtra[ic];
      // ---- copy at the path's last distance (short code 0): run length from the cache
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
      uint32_t fd = 0, fl = 0;   // forced long copy
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
        // ---- hash matches: the staircase of (distance, length)
        const int nm = bnm[off];
        uint32_t prev_len = 3;
        for (int q = 0; q < nm; q++) {
          const uint64_t m = bmt[off * kMaxMatches + q];
          const uint32_t d = (uint32_t)(m >> 32), L = min((uint32_t)m, limit);
          if (L <= prev_len) continue;
          const float dcost = base + bmc[off * kMaxMatches + q];
          if (L > (uint32_t)kLongCopy) {
            fd = d;
            fl = L;
            const int cc = copy_code(L);
            fc = dcost + (float)kCopyExtra[cc] + cmdc[combine_codes(ic, cc, false)];
            break;
          }
#pragma unroll
          for (int k = 0; k < kChunks; k++) {
            if (64 * k + 63 <= (int)prev_len || 64 * k > (int)L) continue;
            const uint32_t l = 64 * k + lane;
            if (l > prev_len && l <= L) {
              const float c = dcost + cxl[k] + cmdc[combine_codes(ic, ccl[k], false)];
              const int ts = (i + l) % kRing;
              if (c < cost[ts]) {
                cost[ts] = c;
                meta[ts] = pack_node(d, l, 0);
              }
            }
          }
          prev_len = L;
        }
        wave_sync();
        if (!fl && ldlen >= 2) {
#pragma unroll
          for (int k = 0; k < kChunks; k++) {
            if (64 * k > (int)ldlen) continue;
            const uint32_t l = 64 * k + lane;
            if (l >= 2 && l <= ldlen) {
              const int cmd = combine_codes(ic, ccl[k], true);
              const float c = base + cxl[k] + cmdc[cmd] + (cmd < 128 ? 0.f : distc[0]);
              const int ts = (i + l) % kRing;
              if (c < cost[ts]) {
                cost[ts] = c;
                meta[ts] = pack_node(ld, l, 0);
              }
            }
          }
          wave_sync();
        }
      }
      if (fl) {
        // forceful long copy (backward-references-hq.ts:518-533): flush the batch's
        // finished nodes, abandon every pending node, resume at the copy's end
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
  uint32_t pend_len = 0, pend_dist = 0;
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
}

// ---------------------------------------------------------------- 5. assemble, lane per stream
__global__ void assemble_kernel(Job *jobs, int njobs, const Seg *segs, Mb *mbs, const RawCmd *raw, Cmd *cmds) {
  int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= njobs) return;
  Job &jb = jobs[j];
  if (jb.uncompressed) return;
  Cmd *out = cmds + jb.cmd_base;
  int dc[4] = {jb.dc_in[0], jb.dc_in[1], jb.dc_in[2], jb.dc_in[3]};   // {4, 11, 15, 16} at stream start
  uint32_t n = 0, carry = 0;
  for (uint32_t m = 0; m < jb.nmb; m++) {
    Mb &mb = mbs[jb.mb_base + m];
    mb.cmd_first = n;
    for (uint32_t s = mb.first_seg; s < mb.first_seg + mb.nseg; s++) {
      const Seg &sg = segs[s];
      const RawCmd *r = raw + sg.cmd_off;
      for (uint32_t q = 0; q < sg.ncmd; q++) {
        uint32_t ins = r[q].ins + carry, len = r[q].len, d = r[q].dist;
        carry = 0;
        // distance code: short codes 0..3 for the cache, else explicit (d + 15)
        uint32_t dcode;
        if (d == (uint32_t)dc[0]) dcode = 0;
        else if (d == (uint32_t)dc[1]) dcode = 1;
        else if (d == (uint32_t)dc[2]) dcode = 2;
        else if (d == (uint32_t)dc[3]) dcode = 3;
        else dcode = d + 15;
        uint32_t extra;
        uint32_t dp = dist_prefix(dcode, (int)jb.ndirect, (int)jb.npostfix, &extra);
        Cmd c;
        c.ins = ins;
        c.copy = len;
        c.dist_extra = extra;
        c.dist_prefix = (uint16_t)dp;
        c.cmd_prefix = (uint16_t)combine_codes(ins_code(ins), copy_code(len), (dp & 0x3FF) == 0);
        out[n++] = c;
        if (dcode > 0) {   // the decoder pushes every distance but code 0 (engine.ts:1361-1364)
          dc[3] = dc[2];
          dc[2] = dc[1];
          dc[1] = dc[0];
          dc[0] = (int)d;
        }
      }
      carry += sg.tail_lits;
    }
    if (carry) {   // trailing literals of the metablock: insert-only command (createInsertCommand)
      Cmd c;
      int ic = ins_code(carry);
      c.ins = carry;
      c.copy = 0;
      c.dist_extra = 0;
      c.dist_prefix = 0;
      c.cmd_prefix = (uint16_t)combine_codes(ic, 0, ic < 8);
      out[n++] = c;
      carry = 0;
    }
    mb.ncmd = n - mb.cmd_first;
  }
  jb.ncmd = n;
  for (int q = 0; q < 4; q++) jb.dc_out[q] = dc[q];
}

// ---------------------------------------------------------------- 6. histograms per metablock
__global__ void histo_kernel(const Job *jobs, const Mb *mbs, int nmbs, const Cmd *cmds, uint32_t *hl, uint32_t *hc,
                             uint32_t *hd) {
  int m = blockIdx.y;
  if (m >= nmbs) return;
  const Mb &mb = mbs[m];
  const Job &jb = jobs[mb.job];
  if (jb.uncompressed) return;
  const Cmd *c = cmds + jb.cmd_base + mb.cmd_first;
  // commands / distances
  for (uint32_t q = blockIdx.x * blockDim.x + threadIdx.x; q < mb.ncmd; q += gridDim.x * blockDim.x) {
    atomicAdd(&hc[m * 704 + c[q].cmd_prefix], 1u);
    if (c[q].copy && c[q].cmd_prefix >= 128) atomicAdd(&hd[m * 128 + (c[q].dist_prefix & 0x3FF)], 1u);
  }
}
// literal histogram: positions that are literals are marked by the segment commands
__global__ void lit_mark_kernel(const Job *jobs, const Mb *mbs, int nmbs, const Cmd *cmds, uint32_t *hl) {
  __shared__ uint32_t h[256];
  int m = blockIdx.x;
  const Mb &mb = mbs[m];
  const Job &jb = jobs[mb.job];
  if (jb.uncompressed) return;
  for (int i = threadIdx.x; i < 256; i += blockDim.x) h[i] = 0;
  __syncthreads();
  const Cmd *c = cmds + jb.cmd_base + mb.cmd_first;
  // each thread walks a strided subset of commands; positions are a prefix sum away, so
  // one serial pass computes the command starts (cheap: O(commands))
  uint32_t pos = mb.start;
  for (uint32_t q = 0; q < mb.ncmd; q++) {
    uint32_t ins = c[q].ins;
    for (uint32_t k = threadIdx.x; k < ins; k += blockDim.x) atomicAdd(&h[jb.data[pos + k]], 1u);
    pos += ins + c[q].copy;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 256; i += blockDim.x) hl[m * 256 + i] = h[i];
}

// ---------------------------------------------------------------- 7. Huffman codes + header
struct BitW {
  uint8_t *buf;
  uint64_t pos;
  __device__ void put(int nbits, uint64_t v) {
    while (nbits > 0) {
      int k = nbits < 32 ? nbits : 32;
      uint64_t vv = v & ((k == 64) ? ~0ull : ((1ull << k) - 1));
      uint64_t p = pos;
      uint64_t word = vv << (p & 7);
      uint8_t *b = buf + (p >> 3);
      int nb = (int)(((p & 7) + k + 7) >> 3);
      for (int i = 0; i < nb; i++) b[i] |= (uint8_t)(word >> (8 * i));
      pos += k;
      v >>= k;
      nbits -= k;
    }
  }
};

// encodeWindowBits (bit-writer.ts:172-194)
__device__ void put_window_bits(BitW &w, int lg) {
  if (lg == 16) w.put(1, 0);
  else if (lg == 17) w.put(7, 1);
  else if (lg > 17) w.put(4, (uint32_t)(((lg - 17) << 1) | 1));
  else w.put(7, (uint32_t)(((lg - 8) << 4) | 1));
}

// createHuffmanTree (entropy-encode.ts:24-131): length-limited depths by count-limit doubling
__device__ void huffman_depths(const uint32_t *h, int len, int limit, uint8_t *depth, uint32_t *cnt, int32_t *left,
                               int32_t *val) {
  for (int i = 0; i < len; i++) depth[i] = 0;
  int nz = 0, last = 0;
  for (int i = 0; i < len; i++)
    if (h[i]) {
      nz++;
      last = i;
    }
  if (nz == 0) return;
  if (nz == 1) {
    depth[last] = 1;
    return;
  }
  for (uint32_t lc = 1;; lc *= 2) {
    int n = 0;
    for (int i = len - 1; i >= 0; i--)
      if (h[i]) {
        cnt[n] = h[i] > lc ? h[i] : lc;
        left[n] = -1;
        val[n] = i;
        n++;
      }
    // insertion sort: count ascending, value descending for ties
    for (int i = 1; i < n; i++) {
      uint32_t tc = cnt[i];
      int32_t tv = val[i];
      int k = i - 1;
      while (k >= 0 && (cnt[k] > tc || (cnt[k] == tc && val[k] < tv))) {
        cnt[k + 1] = cnt[k];
        val[k + 1] = val[k];
        left[k + 1] = left[k];
        k--;
      }
      cnt[k + 1] = tc;
      val[k + 1] = tv;
      left[k + 1] = -1;
    }
    cnt[n] = cnt[n + 1] = 0xFFFFFFFFu;
    left[n] = left[n + 1] = -1;
    val[n] = val[n + 1] = -1;
    int i = 0, jj = n + 1;
    for (int k = n - 1; k > 0; k--) {
      int l, r;
      if (cnt[i] <= cnt[jj]) l = i++; else l = jj++;
      if (cnt[i] <= cnt[jj]) r = i++; else r = jj++;
      int je = 2 * n - k;
      cnt[je] = cnt[l] + cnt[r];
      left[je] = l;
      val[je] = r;
      cnt[je + 1] = 0xFFFFFFFFu;
      left[je + 1] = -1;
      val[je + 1] = -1;
    }
    // depths by an explicit stack walk
    int32_t stack[18];
    int level = 0, p = 2 * n - 1;
    stack[0] = -1;
    bool ok = true;
    for (;;) {
      if (left[p] >= 0) {
        level++;
        if (level > limit) {
          ok = false;
          break;
        }
        stack[level] = val[p];
        p = left[p];
        continue;
      }
      depth[val[p]] = (uint8_t)level;
      while (level >= 0 && stack[level] == -1) level--;
      if (level < 0) break;
      p = stack[level];
      stack[level] = -1;
    }
    if (ok) return;
    for (int q = 0; q < len; q++) depth[q] = 0;
  }
}
__device__ void depths_to_codes(const uint8_t *depth, int len, uint16_t *code) {
  uint32_t bl[16] = {0}, next[16] = {0};
  for (int i = 0; i < len; i++) bl[depth[i]]++;
  bl[0] = 0;
  uint32_t c = 0;
  for (int i = 1; i <= 15; i++) {
    c = (c + bl[i - 1]) << 1;
    next[i] = c;
  }
  for (int i = 0; i < len; i++) {
    if (!depth[i]) continue;
    uint32_t v = next[depth[i]]++, r = 0;
    for (int b = 0; b < depth[i]; b++) r |= ((v >> b) & 1) << (depth[i] - 1 - b);
    code[i] = (uint16_t)r;
  }
}
// buildAndStoreHuffmanTree (context-map.ts:215-347)
__device__ void store_tree(BitW &w, const uint32_t *h, int asize, uint8_t *depth, uint16_t *code, uint32_t *cnt,
                           int32_t *left, int32_t *val) {
  int count = 0, s4[4] = {0, 0, 0, 0};
  for (int i = 0; i < asize; i++)
    if (h[i]) {
      if (count < 4) s4[count] = i;
      count++;
    }
  int max_bits = 0;
  for (int c = asize - 1; c; c >>= 1) max_bits++;
  if (count <= 1) {
    w.put(4, 1);
    w.put(max_bits, (uint32_t)s4[0]);
    for (int i = 0; i < asize; i++) depth[i] = 0, code[i] = 0;
    return;
  }
  huffman_depths(h, asize, 15, depth, cnt, left, val);
  depths_to_codes(depth, asize, code);
  if (count <= 4) {
    int sorted[4];
    for (int i = 0; i < count; i++) sorted[i] = s4[i];
    for (int i = 1; i < count; i++) {
      int t = sorted[i], k = i;
      while (k > 0 && depth[sorted[k - 1]] > depth[t]) {
        sorted[k] = sorted[k - 1];
        k--;
      }
      sorted[k] = t;
    }
    w.put(2, 1);
    w.put(2, (uint32_t)(count - 1));
    for (int i = 0; i < count; i++) w.put(max_bits, (uint32_t)sorted[i]);
    if (count == 4) w.put(1, depth[sorted[0]] == 1 ? 1 : 0);
    return;
  }
  // complex tree: run-length code the depths (codes 16 / 17), then a depth-5 code for them
  uint8_t rle_code[720];
  uint8_t rle_extra[720];
  int nr = 0;
  int nl = asize;
  while (nl > 0 && depth[nl - 1] == 0) nl--;
  int prev = 8;
  for (int i = 0; i < nl;) {
    int v = depth[i], reps = 1;
    while (i + reps < nl && depth[i + reps] == v) reps++;
    i += reps;
    if (v == 0) {
      if (reps == 11) {
        rle_code[nr] = 0; rle_extra[nr++] = 0;
        reps--;
      }
      if (reps < 3) {
        for (int q = 0; q < reps; q++) { rle_code[nr] = 0; rle_extra[nr++] = 0; }
      } else {
        int s0 = nr;
        reps -= 3;
        for (;;) {
          rle_code[nr] = 17; rle_extra[nr++] = (uint8_t)(reps & 7);
          reps >>= 3;
          if (!reps) break;
          reps--;
        }
        for (int x = s0, y = nr - 1; x < y; x++, y--) {
          uint8_t t = rle_code[x]; rle_code[x] = rle_code[y]; rle_code[y] = t;
          t = rle_extra[x]; rle_extra[x] = rle_extra[y]; rle_extra[y] = t;
        }
      }
    } else {
      if (prev != v) { rle_code[nr] = (uint8_t)v; rle_extra[nr++] = 0; reps--; }
      if (reps == 7) { rle_code[nr] = (uint8_t)v; rle_extra[nr++] = 0; reps--; }
      if (reps < 3) {
        for (int q = 0; q < reps; q++) { rle_code[nr] = (uint8_t)v; rle_extra[nr++] = 0; }
      } else {
        int s0 = nr;
        reps -= 3;
        for (;;) {
          rle_code[nr] = 16; rle_extra[nr++] = (uint8_t)(reps & 3);
          reps >>= 2;
          if (!reps) break;
          reps--;
        }
        for (int x = s0, y = nr - 1; x < y; x++, y--) {
          uint8_t t = rle_code[x]; rle_code[x] = rle_code[y]; rle_code[y] = t;
          t = rle_extra[x]; rle_extra[x] = rle_extra[y]; rle_extra[y] = t;
        }
      }
      prev = v;
    }
  }
  uint32_t clh[18] = {0};
  for (int k = 0; k < nr; k++) clh[rle_code[k]]++;
  int ncodes = 0, first = 0;
  for (int k = 0; k < 18; k++)
    if (clh[k]) {
      if (!ncodes) first = k;
      ncodes++;
    }
  uint8_t cld[18];
  uint16_t clc[18] = {0};
  huffman_depths(clh, 18, 5, cld, cnt, left, val);
  depths_to_codes(cld, 18, clc);
  const int order[18] = {1, 2, 3, 4, 0, 5, 17, 6, 16, 7, 8, 9, 10, 11, 12, 13, 14, 15};
  const uint32_t sym[6] = {0, 7, 3, 2, 1, 15};
  const int blen[6] = {2, 4, 3, 2, 2, 4};
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
  for (int k = 0; k < nr; k++) {
    int c = rle_code[k];
    w.put(cld[c], clc[c]);
    if (c == 16) w.put(2, rle_extra[k]);
    else if (c == 17) w.put(3, rle_extra[k]);
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

struct Codes {   // per metablock Huffman codes (device)
  uint8_t ld[256];
  uint16_t lc[256];
  uint8_t cd[704];
  uint16_t cc[704];
  uint8_t dd[128];
  uint16_t dcd[128];
};

// One thread per metablock: window header (first metablock), metablock header, the three
// trees (storeMetaBlockTrivial layout, metablock.ts:290-356); header bits go to hdr.
__global__ void huffman_kernel(Job *jobs, Mb *mbs, int nmbs, const uint32_t *hl, const uint32_t *hc, const uint32_t *hd,
                               Codes *codes, uint8_t *hdr /* 4 KiB per metablock */, uint32_t *work) {
  int m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= nmbs) return;
  Mb &mb = mbs[m];
  Job &jb = jobs[mb.job];
  if (jb.uncompressed) return;
  uint8_t *hb = hdr + (uint64_t)m * 4096;
  for (int i = 0; i < 4096; i++) hb[i] = 0;
  BitW w{hb, 0};
  uint32_t *cnt = work + (uint64_t)m * (3 * 1500);
  int32_t *left = (int32_t *)(cnt + 1500), *val = (int32_t *)(cnt + 3000);
  if (mb.start == 0 && jb.hdr_lgwin) {   // encodeWindowBits (bit-writer.ts:172-194)
    put_window_bits(w, (int)jb.hdr_lgwin);
  }
  uint32_t length = mb.end - mb.start;
  w.put(1, mb.is_last);
  if (mb.is_last) w.put(1, 0);
  int lg = length == 1 ? 1 : 32 - __clz(length - 1);
  int mn = (lg < 16 ? 16 : lg + 3) / 4;
  w.put(2, (uint32_t)(mn - 4));
  w.put(mn * 4, length - 1);
  if (!mb.is_last) w.put(1, 0);
  put_varlen_u8(w, 0);
  put_varlen_u8(w, 0);
  put_varlen_u8(w, 0);
  w.put(2, jb.npostfix);
  w.put(4, jb.ndirect >> jb.npostfix);
  put_varlen_u8(w, 0);
  w.put(2, 0);   // literal context mode LSB6 (one tree: contexts unused)
  put_varlen_u8(w, 0);
  Codes &cd = codes[m];
  int dist_asize = 16 + (int)jb.ndirect + (48 << jb.npostfix);
  store_tree(w, hl + m * 256, 256, cd.ld, cd.lc, cnt, left, val);
  store_tree(w, hc + m * 704, 704, cd.cd, cd.cc, cnt, left, val);
  store_tree(w, hd + m * 128, dist_asize, cd.dd, cd.dcd, cnt, left, val);
  mb.hdr_bits = w.pos;
}

// ---------------------------------------------------------------- 8. sizes (per segment bits)
// The commands of metablock m are re-cut at segment granularity for emission: command q
// belongs to the segment holding its first literal / copy byte.
__global__ void seg_cmd_range_kernel(const Job *jobs, const Mb *mbs, int nmbs, const Cmd *cmds, uint32_t *cmd_pos) {
  int m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= nmbs) return;
  const Mb &mb = mbs[m];
  const Job &jb = jobs[mb.job];
  if (jb.uncompressed) return;
  const Cmd *c = cmds + jb.cmd_base + mb.cmd_first;
  uint32_t *cp = cmd_pos + jb.cmd_base + mb.cmd_first;
  uint32_t pos = mb.start;
  for (uint32_t q = 0; q < mb.ncmd; q++) {
    cp[q] = pos;
    pos += c[q].ins + c[q].copy;
  }
}

__device__ __forceinline__ uint32_t cmd_bits(const Codes &cd, const Cmd &c, uint32_t *ins_extra_n, uint32_t *copy_extra_n) {
  int ic = ins_code(c.ins);
  int cc = copy_code(c.copy ? c.copy : 2);
  *ins_extra_n = kInsExtra[ic];
  *copy_extra_n = kCopyExtra[cc];
  return cd.cd[c.cmd_prefix] + kInsExtra[ic] + kCopyExtra[cc];
}

// bits of commands [q0, q1) of a metablock
__global__ void sizes_kernel(Job *jobs, const Mb *mbs, const Seg *segs, int nsegs, const Cmd *cmds, const uint32_t *cmd_pos,
                             const Codes *codes, uint64_t *seg_bits, uint32_t *seg_q0, uint32_t *seg_q1) {
  int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= nsegs) return;
  const Seg &sg = segs[s];
  const Mb &mb = mbs[sg.mb];
  const Job &jb = jobs[sg.job];
  if (jb.uncompressed) {
    seg_bits[s] = 0;
    return;
  }
  const Cmd *c = cmds + jb.cmd_base + mb.cmd_first;
  const uint32_t *cp = cmd_pos + jb.cmd_base + mb.cmd_first;
  // first command starting at or after sg.start (binary search)
  uint32_t lo = 0, hi = mb.ncmd;
  while (lo < hi) {
    uint32_t mid = (lo + hi) / 2;
    if (cp[mid] < sg.start) lo = mid + 1; else hi = mid;
  }
  uint32_t q0 = lo;
  lo = q0;
  hi = mb.ncmd;
  while (lo < hi) {
    uint32_t mid = (lo + hi) / 2;
    if (cp[mid] < sg.end) lo = mid + 1; else hi = mid;
  }
  uint32_t q1 = lo;
  const Codes &cd = codes[sg.mb];
  uint64_t bits = 0;
  for (uint32_t q = q0; q < q1; q++) {
    uint32_t a, b;
    bits += cmd_bits(cd, c[q], &a, &b);
    uint32_t p = cp[q];
    for (uint32_t k = 0; k < c[q].ins; k++) bits += cd.ld[jb.data[p + k]];
    if (c[q].copy && c[q].cmd_prefix >= 128) bits += cd.dd[c[q].dist_prefix & 0x3FF] + (c[q].dist_prefix >> 10);
  }
  seg_bits[s] = bits;
  seg_q0[s] = q0;
  seg_q1[s] = q1;
}

// lane per stream: metablock / segment bit offsets (stream-relative) and total size
__global__ void offsets_kernel(Job *jobs, int njobs, Mb *mbs, Seg *segs, const uint64_t *seg_bits, uint8_t *out) {
  int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= njobs) return;
  Job &jb = jobs[j];
  if (jb.uncompressed) return;
  uint64_t pos = 0;
  for (uint32_t m = 0; m < jb.nmb; m++) {
    Mb &mb = mbs[jb.mb_base + m];
    mb.bit_off = pos;
    pos += mb.hdr_bits;
    for (uint32_t s = mb.first_seg; s < mb.first_seg + mb.nseg; s++) {
      segs[s].bit_off = pos;
      pos += seg_bits[s];
    }
    if (mb.is_last) pos = (pos + 7) & ~7ull;
  }
  uint64_t trailer = pos;
  if (!jb.final_) pos = (pos + 6 + 7) & ~7ull;   // empty metadata block: ISLAST 0, MNIBBLES 0, MSKIPBYTES 0
  // the stored form is never larger than n + 5 bytes per 16 MiB block + window header + tail
  uint64_t stored_bits = 8ull * ((uint64_t)jb.n + 5ull * ((jb.n >> 24) + 1) + 4);
  if (pos > stored_bits || (pos >> 3) + 8 > jb.out_cap) {
    jb.uncompressed = 2;   // emit stored metablocks instead
    for (int q = 0; q < 4; q++) jb.dc_out[q] = jb.dc_in[q];
    return;
  }
  if (!jb.final_) {   // bits 0,1,1,0,0,0 = 6
    uint32_t *w = reinterpret_cast<uint32_t *>(out + jb.out_off);
    uint64_t v = 6ull << (trailer & 31);
    atomicOr(w + (trailer >> 5), (uint32_t)v);
    if ((uint32_t)(v >> 32)) atomicOr(w + (trailer >> 5) + 1, (uint32_t)(v >> 32));
  }
  jb.total_bits = pos;
}

// ---------------------------------------------------------------- 9. emission
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

__global__ void emit_kernel(const Job *jobs, const Mb *mbs, const Seg *segs, int nsegs, const Cmd *cmds, const uint32_t *cmd_pos,
                            const Codes *codes, const uint32_t *seg_q0, const uint32_t *seg_q1, uint8_t *out) {
  int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= nsegs) return;
  const Seg &sg = segs[s];
  const Mb &mb = mbs[sg.mb];
  const Job &jb = jobs[sg.job];
  if (jb.uncompressed) return;
  const Cmd *c = cmds + jb.cmd_base + mb.cmd_first;
  const uint32_t *cp = cmd_pos + jb.cmd_base + mb.cmd_first;
  const Codes &cd = codes[sg.mb];
  uint32_t *words = reinterpret_cast<uint32_t *>(out + jb.out_off);
  Acc a;
  a.init(words, sg.bit_off);
  for (uint32_t q = seg_q0[s]; q < seg_q1[s]; q++) {
    const Cmd &k = c[q];
    uint32_t ine, cpe;
    cmd_bits(cd, k, &ine, &cpe);
    a.put(cd.cd[k.cmd_prefix], cd.cc[k.cmd_prefix]);
    int ic = ins_code(k.ins);
    a.put((int)ine, k.ins - kInsBase[ic]);
    uint32_t clen = k.copy ? k.copy : 2;
    int cc = copy_code(clen);
    a.put((int)cpe, clen - kCopyBase[cc]);
    uint32_t p = cp[q];
    for (uint32_t t = 0; t < k.ins; t++) {
      uint8_t lit = jb.data[p + t];
      a.put(cd.ld[lit], cd.lc[lit]);
    }
    if (k.copy && k.cmd_prefix >= 128) {
      uint32_t dcode = k.dist_prefix & 0x3FF;
      a.put(cd.dd[dcode], cd.dcd[dcode]);
      a.put(k.dist_prefix >> 10, k.dist_extra);
    }
  }
  a.finish();
}

// metablock headers (bit copy of the header buffer into place), lane per metablock
__global__ void headers_kernel(const Job *jobs, const Mb *mbs, int nmbs, const uint8_t *hdr, uint8_t *out) {
  int m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= nmbs) return;
  const Mb &mb = mbs[m];
  const Job &jb = jobs[mb.job];
  if (jb.uncompressed) return;
  uint32_t *words = reinterpret_cast<uint32_t *>(out + jb.out_off);
  Acc a;
  a.init(words, mb.bit_off);
  const uint8_t *hb = hdr + (uint64_t)m * 4096;
  uint64_t nbits = mb.hdr_bits;
  uint64_t i = 0;
  for (; i + 8 <= nbits; i += 8) a.put(8, hb[i >> 3]);
  if (i < nbits) a.put((int)(nbits - i), hb[i >> 3]);
  a.finish();
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

}  // namespace enc
}  // namespace mib

// ====================================================================== host orchestration
using namespace mib;
using namespace mib::enc;

extern "C" mib_ctx *mib_default_ctx(void);
extern "C" void *mib_ctx_stream_of(mib_ctx *c);
extern "C" int mib_ctx_device_of(mib_ctx *c);
extern "C" void mib_ctx_clear_times(mib_ctx *c);

namespace {

#define CK(x)                                                                                         \
  do {                                                                                                \
    hipError_t e_ = (x);                                                                              \
    if (e_ != hipSuccess) {                                                                           \
      fprintf(stderr, "brotli_amd encode: %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      return MIB_E_NO_DEVICE;                                                                         \
    }                                                                                                 \
  } while (0)

struct Workspace {
  size_t cap = 0;
  uint8_t *buf = nullptr;
};

struct Arena {
  uint8_t *base;
  size_t off = 0;
  template <class T>
  T *take(size_t n) {
    off = (off + 255) & ~(size_t)255;
    T *p = reinterpret_cast<T *>(base + off);
    off += sizeof(T) * std::max<size_t>(n, 1);
    return p;
  }
};

// candidates examined per position (the reference's tree depth / chain length by quality:
// hash-binary-tree.ts:60 maxTreeSearchDepth 64 at q11, 16 at q10; hash-chain.ts by quality)
int depth_for_quality(int q) {
  if (q >= 11) return 64;
  if (q == 10) return 32;
  if (q >= 5) return 16;
  if (q >= 2) return 4;
  return 1;
}

struct Timer {
  mib_ctx *c;
  hipStream_t s;
  bool on;
  std::vector<std::pair<const char *, std::pair<hipEvent_t, hipEvent_t>>> ev;
  void start(const char *name) {
    if (!on) return;
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipEventRecord(a, s);
    ev.push_back({name, {a, b}});
  }
  void stop() {
    if (on) hipEventRecord(ev.back().second.second, s);
  }
  void collect() {
    for (auto &e : ev) {
      float ms = 0;
      hipEventElapsedTime(&ms, e.second.first, e.second.second);
      mib_ctx_add_time(c, e.first, ms);
      hipEventDestroy(e.second.first);
      hipEventDestroy(e.second.second);
    }
    ev.clear();
  }
};

// One stream of a call: where its bytes are and how it is framed.
struct StreamDesc {
  const uint8_t *d_data;
  uint64_t n;
  uint32_t hdr_lgwin;
  uint32_t final_;
  int32_t dc[4];
};

struct Params {
  int quality, lgwin, npostfix, ndirect;
};

Params make_params(const mib_enc_opts *o) {
  Params p;
  p.quality = std::max(0, std::min(11, o ? o->quality : 11));
  p.lgwin = std::max(10, std::min(24, o ? o->lgwin : 22));
  p.npostfix = 0;
  p.ndirect = 0;
  if (p.quality >= 4 && o && o->mode == MIB_MODE_FONT) {   // sanitizeParams (enc-constants.ts:117-127)
    p.npostfix = 1;
    p.ndirect = 12;
  }
  return p;
}

// Encode a group of streams into d_out (packed from out_pos; returns the per-stream sizes).
int encode_group(mib_ctx *ctx, const Params &prm, const StreamDesc *sd, size_t k, uint8_t *d_out, uint64_t out_cap,
                 uint64_t out_pos, uint64_t *sizes, int32_t (*dc_out)[4], hipStream_t st) {
  std::vector<Job> jobs(k);
  std::vector<Seg> segs;
  std::vector<Mb> mbs;
  std::vector<uint32_t> seg_job;
  uint64_t pos_total = 0, cmd_total = 0, out_scratch = 0;
  for (size_t j = 0; j < k; j++) {
    Job &jb = jobs[j];
    memset(&jb, 0, sizeof(jb));
    uint64_t n = sd[j].n;
    jb.data = sd[j].d_data;
    jb.n = (uint32_t)n;
    jb.lgwin = (uint32_t)prm.lgwin;
    jb.npostfix = (uint32_t)prm.npostfix;
    jb.ndirect = (uint32_t)prm.ndirect;
    jb.uncompressed = (prm.quality == 0 || n < 64) ? 1 : 0;
    jb.hdr_lgwin = sd[j].hdr_lgwin;
    jb.final_ = sd[j].final_;
    for (int q = 0; q < 4; q++) jb.dc_in[q] = jb.dc_out[q] = sd[j].dc[q];
    jb.pos_base = (uint32_t)pos_total;
    jb.seg_base = (uint32_t)segs.size();
    jb.mb_base = (uint32_t)mbs.size();
    jb.cmd_base = (uint32_t)cmd_total;
    if (!jb.uncompressed) {
      for (uint64_t m0 = 0; m0 < n; m0 += kMaxMetablock) {
        Mb mb;
        memset(&mb, 0, sizeof(mb));
        mb.job = (uint32_t)j;
        mb.start = (uint32_t)m0;
        mb.end = (uint32_t)std::min<uint64_t>(n, m0 + kMaxMetablock);
        mb.first_seg = (uint32_t)segs.size();
        mb.is_last = (mb.end == n && jb.final_) ? 1 : 0;
        for (uint64_t s0 = m0; s0 < mb.end; s0 += kSeg) {
          Seg sg;
          memset(&sg, 0, sizeof(sg));
          sg.job = (uint32_t)j;
          sg.start = (uint32_t)s0;
          sg.end = (uint32_t)std::min<uint64_t>(mb.end, s0 + kSeg);
          sg.mb = (uint32_t)mbs.size();
          segs.push_back(sg);
        }
        mb.nseg = (uint32_t)segs.size() - mb.first_seg;
        mbs.push_back(mb);
      }
    }
    jb.nseg = (uint32_t)segs.size() - jb.seg_base;
    jb.nmb = (uint32_t)mbs.size() - jb.mb_base;
    uint64_t span = ((n + kSeg - 1) / kSeg) * kSeg + kSeg;   // + a spare segment: end node, padding
    for (uint64_t q = 0; q < span / kSeg; q++) seg_job.push_back((uint32_t)j);
    pos_total += span;
    cmd_total += n / 2 + jb.nmb + 4;
    jb.out_off = out_scratch;
    jb.out_cap = n + n / 8 + 4096;
    out_scratch += (jb.out_cap + 255) & ~255ull;
  }
  if (pos_total >= (1ull << 31)) return MIB_E_INVALID_ARG;
  uint64_t raw_total = 0;
  for (auto &sg : segs) {
    sg.cmd_off = (uint32_t)raw_total;
    raw_total += (sg.end - sg.start) / 2 + 2;
  }
  const uint32_t total = (uint32_t)pos_total;
  const int nsegs = (int)segs.size(), nmbs = (int)mbs.size();
  const size_t nm1 = std::max<size_t>(1, mbs.size()), ns1 = std::max<size_t>(1, segs.size());

  size_t sort_tmp = 0;
  CK(hipcub::DeviceRadixSort::SortPairs(nullptr, sort_tmp, (uint32_t *)nullptr, (uint32_t *)nullptr, (uint32_t *)nullptr,
                                        (uint32_t *)nullptr, (int)total, 0, 32, st));
  size_t need = 64 * 256;
  need += 5 * (size_t)total * 4 + sort_tmp;
  need += (size_t)total * kMaxMatches * 8 + total;
  need += ((size_t)total + 1) * 8;
  need += raw_total * sizeof(RawCmd) + cmd_total * (sizeof(Cmd) + 4);
  need += k * (sizeof(Job) + 1024 + 8) + ns1 * (sizeof(Seg) + 16) + seg_job.size() * 4;
  need += nm1 * (sizeof(Mb) + sizeof(Codes) + 4096 + 4 * (256 + 704 + 128) + 4500 * 4);
  need += out_scratch + 64;
  need += 40 * 256;   // alignment
  Workspace *ws = reinterpret_cast<Workspace *>(*mib_ctx_enc_ws(ctx));
  if (!ws) {
    ws = new Workspace();
    *mib_ctx_enc_ws(ctx) = ws;
  }
  if (ws->cap < need) {
    if (ws->buf) hipFree(ws->buf);
    ws->buf = nullptr;
    ws->cap = 0;
    size_t c = need + need / 8;
    if (hipMalloc(&ws->buf, c) != hipSuccess) return MIB_E_OUT_OF_MEMORY;
    ws->cap = c;
  }
  Arena ar{ws->buf};
  uint32_t *keys = ar.take<uint32_t>(total), *vals = ar.take<uint32_t>(total);
  uint32_t *skeys = ar.take<uint32_t>(total), *svals = ar.take<uint32_t>(total);
  void *sort_ws = ar.take<uint8_t>(sort_tmp);
  uint64_t *matches = ar.take<uint64_t>((size_t)total * kMaxMatches);
  uint8_t *nmatch = ar.take<uint8_t>(total);
  uint64_t *choice = ar.take<uint64_t>((size_t)total + 1);
  RawCmd *raw = ar.take<RawCmd>(raw_total);
  Cmd *cmds = ar.take<Cmd>(cmd_total);
  uint32_t *cmd_pos = ar.take<uint32_t>(cmd_total);
  Job *d_jobs = ar.take<Job>(k);
  Seg *d_segs = ar.take<Seg>(ns1);
  Mb *d_mbs = ar.take<Mb>(nm1);
  uint32_t *d_seg_job = ar.take<uint32_t>(seg_job.size());
  uint32_t *lit_h = ar.take<uint32_t>(k * 256);
  uint32_t *hl = ar.take<uint32_t>(nm1 * 256);
  uint32_t *hc = ar.take<uint32_t>(nm1 * 704);
  uint32_t *hd = ar.take<uint32_t>(nm1 * 128);
  Codes *codes = ar.take<Codes>(nm1);
  uint8_t *hdr = ar.take<uint8_t>(nm1 * 4096);
  uint32_t *hwork = ar.take<uint32_t>(nm1 * 4500);
  uint64_t *seg_bits = ar.take<uint64_t>(ns1);
  uint32_t *seg_q0 = ar.take<uint32_t>(ns1), *seg_q1 = ar.take<uint32_t>(ns1);
  uint64_t *d_dst_off = ar.take<uint64_t>(k + 1);
  uint8_t *oscr = ar.take<uint8_t>(out_scratch + 64);
  if (ar.off > ws->cap) return MIB_E_OUT_OF_MEMORY;

  Timer tm{ctx, st, mib_ctx_profiling(ctx) != 0, {}};
  CK(hipMemcpyAsync(d_jobs, jobs.data(), sizeof(Job) * k, hipMemcpyHostToDevice, st));
  if (nsegs) CK(hipMemcpyAsync(d_segs, segs.data(), sizeof(Seg) * nsegs, hipMemcpyHostToDevice, st));
  if (nmbs) CK(hipMemcpyAsync(d_mbs, mbs.data(), sizeof(Mb) * nmbs, hipMemcpyHostToDevice, st));
  CK(hipMemcpyAsync(d_seg_job, seg_job.data(), seg_job.size() * 4, hipMemcpyHostToDevice, st));
  CK(hipMemsetAsync(oscr, 0, out_scratch + 64, st));
  if (nsegs) {
    CK(hipMemsetAsync(lit_h, 0, k * 256 * 4, st));
    CK(hipMemsetAsync(hl, 0, nm1 * 256 * 4, st));
    CK(hipMemsetAsync(hc, 0, nm1 * 704 * 4, st));
    CK(hipMemsetAsync(hd, 0, nm1 * 128 * 4, st));
    CK(hipMemsetAsync(choice, 0, ((size_t)total + 1) * 8, st));
    const int depth = depth_for_quality(prm.quality);
    const unsigned pgrid = (unsigned)std::min<uint64_t>(8192, (total + 255) / 256);
    tm.start("hash_keys");
    hipLaunchKernelGGL(hash_keys_kernel, dim3(pgrid), dim3(256), 0, st, d_jobs, d_seg_job, total, keys, vals);
    tm.stop();
    tm.start("radix_sort");
    CK(hipcub::DeviceRadixSort::SortPairs(sort_ws, sort_tmp, keys, skeys, vals, svals, (int)total, 0, 32, st));
    tm.stop();
    tm.start("find_matches");
    hipLaunchKernelGGL(find_matches_kernel, dim3((total + kTile - 1) / kTile), dim3(kTile), 0, st, d_jobs, skeys, svals,
                       total, depth, matches, nmatch);
    tm.stop();
    tm.start("lit_histo");
    hipLaunchKernelGGL(lit_histo_kernel, dim3(nsegs), dim3(256), 0, st, d_jobs, d_segs, lit_h);
    tm.stop();
    tm.start("dp_parse");
    hipLaunchKernelGGL(dp_kernel, dim3(nsegs), dim3(64), 0, st, d_jobs, d_segs, lit_h, matches, nmatch, choice);
    tm.stop();
    tm.start("backtrack");
    hipLaunchKernelGGL(backtrack_kernel, dim3((nsegs + 63) / 64), dim3(64), 0, st, d_jobs, d_segs, nsegs, choice, raw);
    tm.stop();
    tm.start("assemble");
    hipLaunchKernelGGL(assemble_kernel, dim3(((int)k + 63) / 64), dim3(64), 0, st, d_jobs, (int)k, d_segs, d_mbs, raw, cmds);
    tm.stop();
    tm.start("histograms");
    hipLaunchKernelGGL(histo_kernel, dim3(64, nmbs), dim3(256), 0, st, d_jobs, d_mbs, nmbs, cmds, hl, hc, hd);
    hipLaunchKernelGGL(lit_mark_kernel, dim3(nmbs), dim3(256), 0, st, d_jobs, d_mbs, nmbs, cmds, hl);
    tm.stop();
    tm.start("huffman");
    hipLaunchKernelGGL(huffman_kernel, dim3((nmbs + 63) / 64), dim3(64), 0, st, d_jobs, d_mbs, nmbs, hl, hc, hd, codes, hdr,
                       hwork);
    tm.stop();
    tm.start("sizes");
    hipLaunchKernelGGL(seg_cmd_range_kernel, dim3((nmbs + 63) / 64), dim3(64), 0, st, d_jobs, d_mbs, nmbs, cmds, cmd_pos);
    hipLaunchKernelGGL(sizes_kernel, dim3((nsegs + 63) / 64), dim3(64), 0, st, d_jobs, d_mbs, d_segs, nsegs, cmds, cmd_pos,
                       codes, seg_bits, seg_q0, seg_q1);
    hipLaunchKernelGGL(offsets_kernel, dim3(((int)k + 63) / 64), dim3(64), 0, st, d_jobs, (int)k, d_mbs, d_segs, seg_bits,
                       oscr);
    tm.stop();
    tm.start("emit");
    hipLaunchKernelGGL(headers_kernel, dim3((nmbs + 63) / 64), dim3(64), 0, st, d_jobs, d_mbs, nmbs, hdr, oscr);
    hipLaunchKernelGGL(emit_kernel, dim3((nsegs + 63) / 64), dim3(64), 0, st, d_jobs, d_mbs, d_segs, nsegs, cmds, cmd_pos,
                       codes, seg_q0, seg_q1, oscr);
    tm.stop();
  }
  tm.start("stored");
  hipLaunchKernelGGL(uncompressed_kernel, dim3((unsigned)k), dim3(256), 0, st, d_jobs, (int)k, oscr);
  tm.stop();
  CK(hipGetLastError());
  CK(hipMemcpyAsync(jobs.data(), d_jobs, sizeof(Job) * k, hipMemcpyDeviceToHost, st));
  CK(hipStreamSynchronize(st));
  std::vector<uint64_t> dst(k + 1);
  dst[0] = out_pos;
  for (size_t j = 0; j < k; j++) {
    uint64_t nb = (jobs[j].total_bits + 7) >> 3;
    if (nb > jobs[j].out_cap) return MIB_E_NO_PROGRESS;   // cannot happen: offsets_kernel falls back first
    sizes[j] = nb;
    dst[j + 1] = dst[j] + nb;
    if (dc_out)
      for (int q = 0; q < 4; q++) dc_out[j][q] = jobs[j].dc_out[q];
  }
  if (dst[k] > out_cap) return MIB_E_NEED_SPACE;
  CK(hipMemcpyAsync(d_dst_off, dst.data(), sizeof(uint64_t) * (k + 1), hipMemcpyHostToDevice, st));
  tm.start("pack");
  hipLaunchKernelGGL(pack_kernel, dim3(64, (unsigned)k), dim3(256), 0, st, d_jobs, d_dst_off, oscr, d_out);
  tm.stop();
  CK(hipGetLastError());
  CK(hipStreamSynchronize(st));
  tm.collect();
  return 0;
}

// workspace bytes per input byte are ~90: groups of at most this many positions
constexpr uint64_t kGroupPositions = 1ull << 28;
constexpr size_t kGroupStreams = 16384;   // job index must fit the 15-bit key field

// Split k streams into groups and encode them back to back into d_out.
int encode_streams(mib_ctx *ctx, const mib_enc_opts *o, const StreamDesc *sd, size_t k, uint8_t *d_out,
                   uint64_t out_cap, uint64_t *out_offsets, int32_t (*dc_out)[4], hipStream_t st) {
  Params prm = make_params(o);
  out_offsets[0] = 0;
  size_t i = 0;
  std::vector<uint64_t> sizes;
  while (i < k) {
    size_t j = i;
    uint64_t pos = 0;
    while (j < k && j - i < kGroupStreams) {
      uint64_t span = ((sd[j].n + kSeg - 1) / kSeg + 1) * kSeg;
      if (j > i && pos + span > kGroupPositions) break;
      pos += span;
      j++;
    }
    sizes.assign(j - i, 0);
    int rc = encode_group(ctx, prm, sd + i, j - i, d_out, out_cap, out_offsets[i], sizes.data(), dc_out ? dc_out + i : nullptr,
                          st);
    if (rc) return rc;
    for (size_t q = i; q < j; q++) out_offsets[q + 1] = out_offsets[q] + sizes[q - i];
    i = j;
  }
  return 0;
}

void fill_desc(StreamDesc &d, const uint8_t *p, uint64_t n, const Params &prm, bool one_shot) {
  d.d_data = p;
  d.n = n;
  d.final_ = 1;
  d.dc[0] = 4;
  d.dc[1] = 11;
  d.dc[2] = 15;
  d.dc[3] = 16;
  if (!one_shot) {
    d.hdr_lgwin = (uint32_t)prm.lgwin;
  } else if (n == 0) {
    d.hdr_lgwin = 10;   // encodeEmptyInput (encode.ts:92-103)
  } else if (prm.quality == 0 || n < 64) {   // encodeUncompressed (encode.ts:105-138)
    int lg = 10;
    if (n > 1) {
      int c = 0;
      while ((1ull << c) < n) c++;
      lg = std::max(10, std::min(24, c + 1));
    }
    d.hdr_lgwin = (uint32_t)lg;
  } else {
    d.hdr_lgwin = (uint32_t)prm.lgwin;
  }
}

uint64_t out_bound(uint64_t n) { return n + n / 8 + 4096; }

}  // namespace

struct mib_encoder {
  mib_enc_opts opts;
  std::vector<uint8_t> pending;
  bool started = false;
  bool finished = false;
  int32_t dc[4] = {4, 11, 15, 16};
  uint64_t block = 1 << 16;
};

extern "C" {

void mib_encode_ws_free(void *p) {
  Workspace *ws = reinterpret_cast<Workspace *>(p);
  if (!ws) return;
  if (ws->buf) hipFree(ws->buf);
  delete ws;
}

int mib_ctx_encode(mib_ctx *c, const mib_enc_opts *o, const uint8_t *d_in, const uint64_t *in_offsets, size_t k,
                   uint8_t *d_out, uint64_t out_cap, uint64_t *out_offsets, void *stream) {
  if (!c || !out_offsets || (k && (!d_in || !in_offsets || !d_out))) return MIB_E_INVALID_ARG;
  if (!mib_default_ctx()) return MIB_E_NO_DEVICE;   // device checks + tables
  CK(hipSetDevice(mib_ctx_device_of(c)));
  hipStream_t st = stream ? (hipStream_t)stream : (hipStream_t)mib_ctx_stream_of(c);
  mib_ctx_clear_times(c);
  Params prm = make_params(o);
  std::vector<StreamDesc> sd(k);
  for (size_t i = 0; i < k; i++) {
    if (in_offsets[i + 1] < in_offsets[i] || in_offsets[i + 1] - in_offsets[i] >= (1ull << 31)) return MIB_E_INVALID_ARG;
    fill_desc(sd[i], d_in + in_offsets[i], in_offsets[i + 1] - in_offsets[i], prm, true);
  }
  return encode_streams(c, o, sd.data(), k, d_out, out_cap, out_offsets, nullptr, st);
}

// host buffers -> device -> encode -> host
static int encode_host(const mib_span *in, size_t k, const mib_enc_opts *o, mib_buf *out, int *status,
                       mib_encoder *streaming, bool final_) {
  mib_ctx *c = mib_default_ctx();
  if (!c) return MIB_E_NO_DEVICE;
  CK(hipSetDevice(mib_ctx_device_of(c)));
  hipStream_t st = (hipStream_t)mib_ctx_stream_of(c);
  Params prm = make_params(o);
  std::vector<uint64_t> ioff(k + 1, 0);
  uint64_t cap = 0;
  for (size_t i = 0; i < k; i++) {
    ioff[i + 1] = ioff[i] + ((in[i].size + 255) & ~(uint64_t)255);
    cap += out_bound(in[i].size);
  }
  uint8_t *d_in = nullptr, *d_out = nullptr;
  if (hipMalloc(&d_in, ioff[k] + 64) != hipSuccess) return MIB_E_OUT_OF_MEMORY;
  if (hipMalloc(&d_out, cap + 64) != hipSuccess) {
    hipFree(d_in);
    return MIB_E_OUT_OF_MEMORY;
  }
  hipMemsetAsync(d_in, 0, ioff[k] + 64, st);
  for (size_t i = 0; i < k; i++)
    if (in[i].size) hipMemcpyAsync(d_in + ioff[i], in[i].data, in[i].size, hipMemcpyHostToDevice, st);
  std::vector<StreamDesc> sd(k);
  for (size_t i = 0; i < k; i++) {
    fill_desc(sd[i], d_in + ioff[i], in[i].size, prm, streaming == nullptr);
    if (streaming) {
      sd[i].hdr_lgwin = streaming->started ? 0 : (uint32_t)prm.lgwin;
      sd[i].final_ = final_ ? 1 : 0;
      for (int q = 0; q < 4; q++) sd[i].dc[q] = streaming->dc[q];
    }
  }
  std::vector<uint64_t> ooff(k + 1, 0);
  std::vector<int32_t> dcs(4 * std::max<size_t>(k, 1));
  int rc = encode_streams(c, o, sd.data(), k, d_out, cap, ooff.data(), (int32_t(*)[4])dcs.data(), st);
  if (rc == 0) {
    std::vector<uint8_t> host(ooff[k]);
    if (ooff[k] && hipMemcpy(host.data(), d_out, ooff[k], hipMemcpyDeviceToHost) != hipSuccess) rc = MIB_E_NO_DEVICE;
    for (size_t i = 0; rc == 0 && i < k; i++) {
      uint64_t len = ooff[i + 1] - ooff[i];
      out[i].data = (uint8_t *)malloc(len ? len : 1);
      out[i].size = len;
      if (len) memcpy(out[i].data, host.data() + ooff[i], len);
      if (status) status[i] = 0;
    }
    if (streaming && k == 1)
      for (int q = 0; q < 4; q++) streaming->dc[q] = dcs[q];
  }
  hipFree(d_out);
  hipFree(d_in);
  return rc;
}

int mib_encode(const uint8_t *in, size_t n, const mib_enc_opts *o, mib_buf *out) {
  if (!out || (!in && n)) return MIB_E_INVALID_ARG;
  out->data = nullptr;
  out->size = 0;
  if (n >= (1ull << 31)) return MIB_E_INVALID_ARG;
  mib_span s{in, n};
  return encode_host(&s, 1, o, out, nullptr, nullptr, true);
}

int mib_encode_batch(const mib_span *in, size_t k, const mib_enc_opts *o, mib_buf *out, int *status) {
  if (k && (!in || !out || !status)) return MIB_E_INVALID_ARG;
  for (size_t i = 0; i < k; i++) {
    out[i].data = nullptr;
    out[i].size = 0;
    status[i] = 0;
    if ((!in[i].data && in[i].size) || in[i].size >= (1ull << 31)) return MIB_E_INVALID_ARG;
  }
  if (!k) return 0;
  return encode_host(in, k, o, out, status, nullptr, true);
}

// BrotliEncoder (encode.ts:290-409): input is cut into blocks of 2^lgblock (computeLgBlock,
// enc-constants.ts:129-147); each full block becomes metablocks ending in a byte-aligning
// empty metadata block, so update() can return whole bytes.  The distance cache carries over.
mib_encoder *mib_encoder_new(const mib_enc_opts *o) {
  mib_encoder *e = new mib_encoder();
  if (o) e->opts = *o;
  else mib_enc_opts_default(&e->opts);
  Params prm = make_params(&e->opts);
  int lgblock;
  if (prm.quality == 0 || prm.quality == 1) lgblock = prm.lgwin;
  else if (prm.quality < 4) lgblock = 14;
  else {
    lgblock = 16;
    if (prm.quality >= 9 && prm.lgwin > lgblock) lgblock = std::min(18, prm.lgwin);
  }
  e->block = 1ull << lgblock;
  return e;
}

static int encoder_emit(mib_encoder *e, const uint8_t *p, size_t n, bool final_, std::vector<uint8_t> &acc) {
  mib_span s{p, n};
  mib_buf b{nullptr, 0};
  int st = 0;
  int rc = encode_host(&s, 1, &e->opts, &b, &st, e, final_);
  if (rc) return rc;
  acc.insert(acc.end(), b.data, b.data + b.size);
  mib_buf_free(&b);
  e->started = true;
  return 0;
}

int mib_encoder_update(mib_encoder *e, const uint8_t *in, size_t n, mib_buf *out) {
  if (!e || !out || (!in && n)) return MIB_E_INVALID_ARG;
  out->data = nullptr;
  out->size = 0;
  if (e->finished) return MIB_E_INVALID_ARG;
  e->pending.insert(e->pending.end(), in, in + n);
  std::vector<uint8_t> acc;
  size_t off = 0;
  while (e->pending.size() - off >= e->block) {
    int rc = encoder_emit(e, e->pending.data() + off, e->block, false, acc);
    if (rc) return rc;
    off += e->block;
  }
  e->pending.erase(e->pending.begin(), e->pending.begin() + off);
  out->data = (uint8_t *)malloc(acc.size() ? acc.size() : 1);
  out->size = acc.size();
  if (acc.size()) memcpy(out->data, acc.data(), acc.size());
  return 0;
}

int mib_encoder_finish(mib_encoder *e, mib_buf *out) {
  if (!e || !out) return MIB_E_INVALID_ARG;
  out->data = nullptr;
  out->size = 0;
  std::vector<uint8_t> acc;
  if (!e->finished) {
    int rc = encoder_emit(e, e->pending.data(), e->pending.size(), true, acc);
    if (rc) return rc;
    e->pending.clear();
    e->finished = true;
  }
  out->data = (uint8_t *)malloc(acc.size() ? acc.size() : 1);
  out->size = acc.size();
  if (acc.size()) memcpy(out->data, acc.data(), acc.size());
  return 0;
}

void mib_encoder_free(mib_encoder *e) { delete e; }

}  // extern "C"
