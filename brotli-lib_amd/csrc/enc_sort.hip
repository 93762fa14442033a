// The bucket sort of the match finder: every position of every
// stream gets an 18-bit key (the hash of its first kHashBytes bytes, or the invalid mark
// kInvalidKey for the padding and a stream's last bytes), and each stream's positions are
// sorted by key, stably -- so every hash bucket of a stream becomes one run of positions in
// ascending order, the candidate chain find_matches walks (the reference's per-bucket binary
// tree / hash chain, hash-binary-tree.ts:57-227, hash-chains.ts:69-153).
//
// Streams occupy disjoint ranges of global positions (64 KiB aligned), so the whole call is a
// segmented sort: two LSD passes of 9-bit digits, each
//   tile_hist  block per 8192-position tile: the tile's digit counts (pass 1 computes the keys
//              from the stream bytes on the fly: no key array is written before the sort)
//   tile_scan  block per stream, thread per digit: each (tile, digit)'s first output slot
//              (the digit's count in the stream's earlier tiles + the stream's earlier digits)
//   scatter    block per tile, wave per quarter: a stable counting sort of the tile in LDS
//              (each wave ranks its 2048 items round by round, 64 at a time, by returning LDS
//              atomics, which serve the lanes of a wave in lane order), then coalesced runs
//              to the output
// Traffic per position: pass 1 reads the bytes twice and writes key + position (8 B), pass 2
// reads the keys (4 B), then key + position, and writes 8 B: ~30 B.  (It replaced a
// library radix sort of (stream group | hash) keys: three 8-bit passes over key + value
// arrays written by a separate key kernel, 24 + 3 ms on C4.)

#include <algorithm>
#include <vector>

#include "enc_common.h"

namespace mib {
namespace enc {

// (the hardware property the ranking relies on, checked by the GPU tests)
__global__ void lds_atomic_order_kernel(const uint32_t *addr, int trials, uint32_t *bad) {
  __shared__ uint32_t cnt[4][64];
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t nbad = 0;
  for (int t = blockIdx.x * 4 + (int)w; t < trials; t += gridDim.x * 4) {
    cnt[w][lane] = 0;
    __builtin_amdgcn_wave_barrier();
    const uint32_t a = addr[t * 64 + lane] & 63;
    const uint32_t r = atomicAdd(&cnt[w][a], 1u);
    __builtin_amdgcn_wave_barrier();
    uint32_t below = 0;
    for (int l = 0; l < 64; l++) {
      const uint32_t al = (uint32_t)__shfl((int)a, l);   // (every lane: a shuffle reads active lanes only)
      below += ((uint32_t)l < lane && al == a) ? 1u : 0u;
    }
    nbad += r != below ? 1u : 0u;
  }
  atomicAdd(bad, nbad);
}

constexpr int kTileBits = 13;
constexpr uint32_t kTile = 1u << kTileBits;   // positions per tile (a stream's span is a multiple)
constexpr int kDigitBits = 9;
constexpr int kDigits = 1 << kDigitBits;
constexpr int kSortT = 256;                   // threads of the tile kernels (4 waves)
constexpr int kPerThread = kTile / kSortT;    // 32
static_assert(2 * kDigitBits >= kHashBits + 1, "two digits cover the key");

// keys of the 4 positions g .. g + 3 (one stream): the hash of hb bytes, kInvalidKey where
// fewer than hb bytes remain (or the stream is stored uncompressed)
__device__ __forceinline__ void keys4(const Job &jb, uint32_t p, int hb, uint32_t *k4) {
  if (!jb.uncompressed && p + 16 <= jb.n) {
    const uintptr_t a = (uintptr_t)(jb.data + p);
    const uint32_t *w = (const uint32_t *)(a & ~(uintptr_t)3);
    const uint32_t sh = (uint32_t)(a & 3);
    const uint32_t v0 = w[0], v1 = w[1], v2 = w[2], v3 = w[3];
    const uint64_t lo = (uint64_t)__builtin_amdgcn_alignbyte(v1, v0, sh) | ((uint64_t)__builtin_amdgcn_alignbyte(v2, v1, sh) << 32);
    const uint64_t hi = __builtin_amdgcn_alignbyte(v3, v2, sh);   // bytes 8..11
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const uint64_t x = k ? (lo >> (8 * k)) | (hi << (64 - 8 * k)) : lo;
      const uint64_t v = (x & ((1ull << (8 * hb)) - 1)) << (64 - 8 * hb);   // (= hashn)
      k4[k] = (uint32_t)((v * 0x1E35A7BD1E35A7BDull) >> (64 - kHashBits));
    }
  } else {
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const uint32_t q = p + k;
      k4[k] = (q + (uint32_t)hb <= jb.n && !jb.uncompressed) ? hashn(jb.data + q, hb) : kInvalidKey;
    }
  }
}

// the tile's items, thread t holding items t * 4 + 1024 k + (0..3), k = 0..7 (so each 16-byte
// load of the stream covers a thread's four positions): pass 1 computes the keys, pass 2 reads
// them (and the positions) from the first pass's output
template <bool kFirst>
__device__ __forceinline__ void load_items(const Job *jobs, const uint32_t *pos_job, uint32_t tile, int hb, const uint32_t *in_k,
                                           const uint32_t *in_v, uint32_t *key, uint32_t *val) {
  const uint32_t base = tile << kTileBits;
#pragma unroll
  for (int k = 0; k < kPerThread / 4; k++) {
    const uint32_t g = base + 1024u * k + 4u * threadIdx.x;
    if (kFirst) {
      const Job &jb = jobs[pos_job[g >> kSegBits]];
      keys4(jb, g - jb.pos_base, hb, key + 4 * k);
#pragma unroll
      for (int q = 0; q < 4; q++) val[4 * k + q] = g + q;
    } else {
      const uint4 kk = *reinterpret_cast<const uint4 *>(in_k + g), vv = *reinterpret_cast<const uint4 *>(in_v + g);
      key[4 * k] = kk.x; key[4 * k + 1] = kk.y; key[4 * k + 2] = kk.z; key[4 * k + 3] = kk.w;
      val[4 * k] = vv.x; val[4 * k + 1] = vv.y; val[4 * k + 2] = vv.z; val[4 * k + 3] = vv.w;
    }
  }
}

template <bool kFirst>
__device__ __forceinline__ uint32_t digit_of(uint32_t key) {
  return kFirst ? key & (kDigits - 1) : key >> kDigitBits;
}

template <bool kFirst>
__global__ __launch_bounds__(kSortT) void tile_hist_kernel(const Job *jobs, const uint32_t *pos_job, int hb, const uint32_t *in_k,
                                                           uint16_t *hist) {
  __shared__ uint32_t h[kDigits];
  for (int d = threadIdx.x; d < kDigits; d += kSortT) h[d] = 0;
  __syncthreads();
  const uint32_t tile = blockIdx.x;
  if (kFirst) {
    uint32_t key[kPerThread], val[kPerThread];
    load_items<true>(jobs, pos_job, tile, hb, nullptr, nullptr, key, val);
#pragma unroll
    for (int i = 0; i < kPerThread; i++) atomicAdd(&h[digit_of<true>(key[i])], 1u);
  } else {
    const uint32_t base = tile << kTileBits;
    for (uint32_t i = threadIdx.x; i < kTile; i += kSortT) atomicAdd(&h[digit_of<false>(in_k[base + i])], 1u);
  }
  __syncthreads();
  for (int d = threadIdx.x; d < kDigits; d += kSortT) hist[(size_t)tile * kDigits + d] = (uint16_t)h[d];
}

// Block per stream, thread per digit: off[tile][d] = the output slot of the tile's first item
// of digit d = pos_base + (items of the stream with a smaller digit) + (items of digit d in
// the stream's earlier tiles).  The tile loop keeps eight loads in flight.
__global__ __launch_bounds__(kDigits) void tile_scan_kernel(const Job *jobs, int njobs, uint32_t total, const uint16_t *hist,
                                                            uint32_t *off) {
  __shared__ uint32_t sc[kDigits];
  const int s = blockIdx.x;
  const uint32_t d = threadIdx.x;
  const uint32_t t0 = jobs[s].pos_base >> kTileBits, t1 = (s + 1 < njobs ? jobs[s + 1].pos_base : total) >> kTileBits;
  uint32_t sum = 0;
  uint32_t t = t0;
  for (; t + 8 <= t1; t += 8) {
    uint32_t c[8];
#pragma unroll
    for (int q = 0; q < 8; q++) c[q] = hist[(size_t)(t + q) * kDigits + d];
#pragma unroll
    for (int q = 0; q < 8; q++) sum += c[q];
  }
  for (; t < t1; t++) sum += hist[(size_t)t * kDigits + d];
  // exclusive scan of the digit totals (Hillis-Steele over the block)
  sc[d] = sum;
  __syncthreads();
  for (uint32_t o = 1; o < kDigits; o <<= 1) {
    const uint32_t v = d >= o ? sc[d - o] : 0u;
    __syncthreads();
    sc[d] += v;
    __syncthreads();
  }
  uint32_t run = jobs[s].pos_base + sc[d] - sum;
  for (t = t0; t + 8 <= t1; t += 8) {
    uint32_t c[8];
#pragma unroll
    for (int q = 0; q < 8; q++) c[q] = hist[(size_t)(t + q) * kDigits + d];
#pragma unroll
    for (int q = 0; q < 8; q++) {
      off[(size_t)(t + q) * kDigits + d] = run;
      run += c[q];
    }
  }
  for (; t < t1; t++) {
    off[(size_t)t * kDigits + d] = run;
    run += hist[(size_t)t * kDigits + d];
  }
}

// Block per tile.  Wave w owns items [2048 w, 2048 (w + 1)) of the tile in position order;
// stable order = wave order, then round order, then lane order.  Sweep 1: each wave's digit
// counts; their prefix over the waves and the tile's digit offsets give each wave its first
// slot per digit.  Sweep 2, round by round: each item takes its digit's next slot (cur) by a
// returning atomic.  Items go to LDS in sorted order, then out in runs.
template <bool kFirst, bool kBallotRank>
__global__ __launch_bounds__(kSortT) void tile_scatter_kernel(const Job *jobs, const uint32_t *pos_job, int hb,
                                                              const uint32_t *in_k, const uint32_t *in_v, const uint16_t *hist,
                                                              const uint32_t *off, uint32_t *out_k, uint32_t *out_v) {
  constexpr int kW = kSortT / 64;
  constexpr int kRounds = kTile / kSortT;   // rounds per wave (64 items each)
  __shared__ uint32_t sk[kTile], sv[kTile];
  __shared__ uint32_t cur[kW][kDigits];     // sweep 1: the wave's counts; sweep 2: its next slot
  __shared__ uint32_t lbase[kDigits];       // the tile's first slot per digit
  __shared__ uint32_t obase[kDigits];       // output index of sorted item i of digit d: obase[d] + i
  const uint32_t tile = blockIdx.x, t = threadIdx.x, lane = t & 63, w = t >> 6;
  const uint32_t base = tile << kTileBits;
  for (uint32_t d = t; d < kDigits; d += kSortT) {
#pragma unroll
    for (int q = 0; q < kW; q++) cur[q][d] = 0;
    lbase[d] = hist[(size_t)tile * kDigits + d];
  }
  __syncthreads();
  // pass 1: the tile's keys, four consecutive positions per thread from one 16-byte load of
  // the stream (load_items), staged in sk in position order
  if (kFirst) {
    uint32_t k4[kPerThread], v4[kPerThread];
    load_items<true>(jobs, pos_job, tile, hb, nullptr, nullptr, k4, v4);
#pragma unroll
    for (int k = 0; k < kPerThread / 4; k++)
#pragma unroll
      for (int q = 0; q < 4; q++) sk[1024 * k + 4 * t + q] = k4[4 * k + q];
    __syncthreads();
  }
  // the wave's items: round r, lane l -> tile item 2048 w + 64 r + l
  uint32_t key[kRounds], val[kRounds];
#pragma unroll
  for (int r = 0; r < kRounds; r++) {
    const uint32_t i = (w << 11) + 64u * r + lane;
    if (kFirst) {
      key[r] = sk[i];
      val[r] = base + i;
    } else {
      key[r] = in_k[base + i];
      val[r] = in_v[base + i];
    }
  }
  // (a loop of its own: with the count in the load loop every load was waited for at once)
#pragma unroll
  for (int r = 0; r < kRounds; r++) atomicAdd(&cur[w][digit_of<kFirst>(key[r])], 1u);
  __syncthreads();
  // lbase: exclusive scan of the tile's digit counts; cur[w][d]: lbase[d] + the counts of the
  // waves before w
  if (t < 64) {   // one wave scans the 512 counts (8 per lane)
    uint32_t c[kDigits / 64], s = 0;
#pragma unroll
    for (int q = 0; q < kDigits / 64; q++) {
      c[q] = lbase[t * (kDigits / 64) + q];
      s += c[q];
    }
    uint32_t incl = s;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = (uint32_t)__shfl_up((int)incl, o);
      if (lane >= (uint32_t)o) incl += y;
    }
    uint32_t run = incl - s;
#pragma unroll
    for (int q = 0; q < kDigits / 64; q++) {
      lbase[t * (kDigits / 64) + q] = run;
      run += c[q];
    }
  }
  __syncthreads();
  for (uint32_t d = t; d < kDigits; d += kSortT) {
    obase[d] = off[(size_t)tile * kDigits + d] - lbase[d];
    uint32_t run = lbase[d];
#pragma unroll
    for (int q = 0; q < kW; q++) {
      const uint32_t c = cur[q][d];
      cur[q][d] = run;
      run += c;
    }
  }
  __syncthreads();
  // Ranking: one returning LDS atomic per item.  The lanes of one ds_add_rtn_u32 that hit the
  // same address get their values in lane order (probed on the MI355X over 65,536 random
  // collision patterns: scripts/probe/lds_atomic_order.hip, and mib_selftest_lds_atomic_order
  // in the GPU tests), and a wave's LDS operations complete in issue order: so round r's items
  // take their digit's slots in (round, lane) order -- the sort is stable.  (Nine ballots per
  // round to the same effect cost ~90 VALU per round: the whole pass was VALU-bound.)
  // kBallotRank: that ballot ranking, which does not depend on the atomics' lane order -- the
  // build runs it on a device whose self-test (ensure_device, runtime.cpp) saw them out of order.
#pragma unroll
  for (int r = 0; r < kRounds; r++) {
    const uint32_t d = digit_of<kFirst>(key[r]);
    uint32_t slot;
    if (kBallotRank) {
      uint64_t m = ~0ull;
#pragma unroll
      for (int b = 0; b < kDigitBits; b++) {
        const uint64_t bb = __ballot((d >> b) & 1u);
        m &= ((d >> b) & 1u) ? bb : ~bb;
      }
      const int leader = __ffsll((unsigned long long)m) - 1;
      uint32_t first = 0;
      if ((int)lane == leader) first = atomicAdd(&cur[w][d], (uint32_t)__popcll(m));
      first = (uint32_t)__shfl((int)first, leader);
      slot = first + (uint32_t)__popcll(m & ((1ull << lane) - 1));
    } else {
      slot = atomicAdd(&cur[w][d], 1u);
    }
    sk[slot] = key[r];
    sv[slot] = val[r];
  }
  __syncthreads();
  // out: item i (sorted) of digit d goes to off[tile][d] + (i - lbase[d]); consecutive threads,
  // consecutive slots within a digit's run
  for (uint32_t i = t; i < kTile; i += kSortT) {
    const uint32_t k = sk[i], d = digit_of<kFirst>(k);
    const uint32_t dst = obase[d] + i;
    out_k[dst] = k;
    out_v[dst] = sv[i];
  }
}

}  // namespace enc
}  // namespace mib

// Self-test: lanes of one wave colliding on LDS addresses through returning atomics (random
// patterns of 1..64 addresses, `trials` of them): how many lanes got a value other than their
// rank in lane order (0 on the MI355X).  Returns that count, or < 0 on a HIP error.
extern "C" int64_t mib_selftest_lds_atomic_order(int trials) {
  if (trials <= 0) return 0;
  std::vector<uint32_t> h((size_t)trials * 64);
  uint32_t x = 12345;
  for (int t = 0; t < trials; t++) {
    const uint32_t range = 1 + (uint32_t)(t % 64);
    for (int l = 0; l < 64; l++) {
      x ^= x << 13; x ^= x >> 17; x ^= x << 5;
      h[(size_t)t * 64 + l] = x % range;
    }
  }
  uint32_t *d = nullptr, *bad = nullptr, nb = 0;
  if (hipMalloc(&d, h.size() * 4) != hipSuccess) return -1;
  if (hipMalloc(&bad, 4) != hipSuccess) {
    hipFree(d);
    return -1;
  }
  int64_t rc = -1;
  if (hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice) == hipSuccess && hipMemset(bad, 0, 4) == hipSuccess) {
    hipLaunchKernelGGL(mib::enc::lds_atomic_order_kernel, dim3(256), dim3(256), 0, 0, d, trials, bad);
    if (hipMemcpy(&nb, bad, 4, hipMemcpyDeviceToHost) == hipSuccess) rc = nb;
  }
  hipFree(d);
  hipFree(bad);
  return rc;
}

namespace mib {
namespace enc {

static uint16_t *hist_of(void *ws) { return reinterpret_cast<uint16_t *>(ws); }
static uint32_t *off_of(void *ws, uint32_t ntiles) {
  return reinterpret_cast<uint32_t *>((uint8_t *)ws + (((size_t)ntiles * kDigits * 2 + 255) & ~(size_t)255));
}

size_t sort_ws_bytes(uint32_t total) {
  const size_t ntiles = total >> kTileBits;
  return ntiles * kDigits * (sizeof(uint16_t) + sizeof(uint32_t)) + 512;
}

void launch_sort(hipStream_t st, const Job *jobs, const uint32_t *pos_job, int njobs, uint32_t total, int hb, void *ws,
                 uint32_t *tmp_k, uint32_t *tmp_v, uint32_t *skeys, uint32_t *svals) {
  const uint32_t ntiles = total >> kTileBits;
  if (!ntiles) return;
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (!lds_rank_ordered(dev)) {   // (the self-test found returning LDS atomics out of lane order)
    hipLaunchKernelGGL(tile_hist_kernel<true>, dim3(ntiles), dim3(kSortT), 0, st, jobs, pos_job, hb, nullptr, hist_of(ws));
    hipLaunchKernelGGL(tile_scan_kernel, dim3(njobs), dim3(kDigits), 0, st, jobs, njobs, total, hist_of(ws), off_of(ws, ntiles));
    hipLaunchKernelGGL((tile_scatter_kernel<true, true>), dim3(ntiles), dim3(kSortT), 0, st, jobs, pos_job, hb, nullptr, nullptr,
                       hist_of(ws), off_of(ws, ntiles), tmp_k, tmp_v);
    hipLaunchKernelGGL(tile_hist_kernel<false>, dim3(ntiles), dim3(kSortT), 0, st, jobs, pos_job, hb, tmp_k, hist_of(ws));
    hipLaunchKernelGGL(tile_scan_kernel, dim3(njobs), dim3(kDigits), 0, st, jobs, njobs, total, hist_of(ws), off_of(ws, ntiles));
    hipLaunchKernelGGL((tile_scatter_kernel<false, true>), dim3(ntiles), dim3(kSortT), 0, st, jobs, pos_job, hb, tmp_k, tmp_v,
                       hist_of(ws), off_of(ws, ntiles), skeys, svals);
    return;
  }
  uint16_t *hist = reinterpret_cast<uint16_t *>(ws);
  uint32_t *off = reinterpret_cast<uint32_t *>((uint8_t *)ws + (((size_t)ntiles * kDigits * 2 + 255) & ~(size_t)255));
  // pass 1: low digit, keys from the stream bytes -> tmp
  hipLaunchKernelGGL(tile_hist_kernel<true>, dim3(ntiles), dim3(kSortT), 0, st, jobs, pos_job, hb, nullptr, hist);
  hipLaunchKernelGGL(tile_scan_kernel, dim3(njobs), dim3(kDigits), 0, st, jobs, njobs, total, hist, off);
  hipLaunchKernelGGL((tile_scatter_kernel<true, false>), dim3(ntiles), dim3(kSortT), 0, st, jobs, pos_job, hb, nullptr, nullptr, hist, off,
                     tmp_k, tmp_v);
  // pass 2: high digit, tmp -> sorted
  hipLaunchKernelGGL(tile_hist_kernel<false>, dim3(ntiles), dim3(kSortT), 0, st, jobs, pos_job, hb, tmp_k, hist);
  hipLaunchKernelGGL(tile_scan_kernel, dim3(njobs), dim3(kDigits), 0, st, jobs, njobs, total, hist, off);
  hipLaunchKernelGGL((tile_scatter_kernel<false, false>), dim3(ntiles), dim3(kSortT), 0, st, jobs, pos_job, hb, tmp_k, tmp_v, hist, off,
                     skeys, svals);
}

}  // namespace enc
}  // namespace mib
