// Match finding: hash keys, the device radix sort that turns
// every hash bucket into a flat chain, and the LDS-tiled candidate walk.
#include <algorithm>

#include "enc_common.h"

namespace mib {
namespace enc {

// ---------------------------------------------------------------- 1. keys
// Every global position (including the padding after each stream) gets the key
// (stream group << 18 | hash4), the invalid hash 2^17 for padding and a stream's last 3
// bytes.  A stream group is 2^gshift consecutive streams (at most 64 groups a call, so keys
// have at most 24 bits: three radix passes).  The sort is stable and global positions
// ascend stream by stream, so within a bucket the entries of one stream are contiguous and
// in position order -- a candidate walk stops where the stream changes -- and the entries a
// wave of find_matches tiles touches stay within one group's streams (cache locality).
__global__ void hash_keys_kernel(const Job *jobs, const uint32_t *pos_job, uint32_t total, int gshift, uint32_t *keys,
                                 uint32_t *vals) {
  for (uint32_t g = blockIdx.x * blockDim.x + threadIdx.x; g < total; g += gridDim.x * blockDim.x) {
    uint32_t j = pos_job[g >> kSegBits];
    const Job &jb = jobs[j];
    uint32_t p = g - jb.pos_base;
    keys[g] = ((j >> gshift) << (kHashBits + 1)) | ((p + 4 <= jb.n && !jb.uncompressed) ? hash4(jb.data + p) : kInvalidKey);
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
  if (avail >= 12) {   // three aligned words (all inside the stream) and two funnel shifts
    const uintptr_t a = (uintptr_t)p;
    const uint32_t *w = (const uint32_t *)(a & ~(uintptr_t)3);
    const uint32_t sh = (uint32_t)(a & 3);
    const uint32_t w0 = w[0], w1 = w[1], w2 = w[2];
    const uint32_t lo = __builtin_amdgcn_alignbyte(w1, w0, sh), hi = __builtin_amdgcn_alignbyte(w2, w1, sh);
    return ((uint64_t)hi << 32) | lo;
  }
  uint64_t v = 0;
  for (uint32_t i = 0; i < avail; i++) v |= (uint64_t)p[i] << (8 * i);
  return v;
}

__global__ __launch_bounds__(kTile) void find_matches_kernel(const Job *jobs, const uint32_t *pos_job, const uint32_t *sorted_keys,
                                                             const uint32_t *sorted_vals, uint32_t total, int depth,
                                                             uint32_t *matches) {
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
      if ((key & kInvalidKey) == 0) {
        const Job &jb = jobs[pos_job[g >> kSegBits]];
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
  if ((key & kInvalidKey) == 0) {
    const Job &jb = jobs[pos_job[g >> kSegBits]];
    const uint32_t p = g - jb.pos_base;
    const uint32_t max_dist = (1u << jb.lgwin) - 16;
    const uint32_t seg_end = min(((p >> kSegBits) + 1) << kSegBits, jb.n);
    const uint32_t limit = seg_end - p;   // copies never cross a parse segment
    const uint8_t *cur = jb.data + p;
    const uint64_t mine = spre[me];
    uint32_t best = 3;
    uint32_t local[kMaxMatches] = {0u, 0u, 0u, 0u};
    const int dmax = min(depth, kBack);
    for (int t = 1; t <= dmax; t++) {
      const int e = me - t;
      if (skey[e] != key || spos[e] < jb.pos_base) break;   // bucket or stream changes
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
        // measured up to the saturation length: the parse measures longer copies itself
        const uint32_t lim = min(limit, kMatchLenSat);
        len = 8 + match_len(cur + 8, cand + 8, lim > 8 ? lim - 8 : 0);
        len = min(len, limit);
      }
      if (len > best) {
        best = len;
        if (cnt == kMaxMatches) {   // keep the longest ones: drop the shortest
          for (int q = 1; q < kMaxMatches; q++) local[q - 1] = local[q];
          cnt--;
        }
        local[cnt++] = pack_match(d, len);
        if (len >= limit || len >= kMatchLenSat) break;   // the parse measures a long copy itself
      }
    }
    // a match word is never 0 (length >= 4): the unused tail entries mark the count
    *reinterpret_cast<uint4 *>(matches + (uint64_t)g * kMatchRec) = make_uint4(local[0], local[1], local[2], local[3]);
    return;
  }
  *reinterpret_cast<uint4 *>(matches + (uint64_t)g * kMatchRec) = make_uint4(0u, 0u, 0u, 0u);   // no candidates
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


void launch_hash_keys(hipStream_t st, const Job *jobs, const uint32_t *pos_job, uint32_t total, int gshift, uint32_t *keys,
                      uint32_t *vals) {
  const unsigned grid = (unsigned)std::min<uint64_t>(8192, (total + 255) / 256);
  hipLaunchKernelGGL(hash_keys_kernel, dim3(grid), dim3(256), 0, st, jobs, pos_job, total, gshift, keys, vals);
}
void launch_find_matches(hipStream_t st, const Job *jobs, const uint32_t *pos_job, const uint32_t *skeys,
                         const uint32_t *svals, uint32_t total, int depth, uint32_t *matches) {
  hipLaunchKernelGGL(find_matches_kernel, dim3((total + kTile - 1) / kTile), dim3(kTile), 0, st, jobs, pos_job, skeys, svals,
                     total, depth, matches);
}
void launch_lit_histo(hipStream_t st, const Job *jobs, const Seg *segs, int nsegs, uint32_t *lit_h) {
  hipLaunchKernelGGL(lit_histo_kernel, dim3(nsegs), dim3(256), 0, st, jobs, segs, lit_h);
}

}  // namespace enc
}  // namespace mib
