// Traffic calibration probe: read patterns with a known number of
// accesses, each to its own memory line of a buffer far larger than L2 + Infinity Cache, so
// every access misses to HBM.  rocprofv3 --pmc FETCH_SIZE (and the EA request counters) on
// this program gives the counters' bytes per access for each access width; the ratio to the
// algorithmic bytes calibrates the traffic figures of the engine's gather-bound kernels
// (decoder: byte loads and LDS-DMA byte gathers; find_matches: 36-byte prefix gathers).
//
// Kernels (one launch each, in this order; names carry the pattern):
//   probe_stream16   16 B per lane, coalesced, over the whole buffer (the guide's calibrated case)
//   probe_gather1    1 B per access at a random distinct 256 B-aligned line
//   probe_gather4    4 B (one dword)
//   probe_gather16   16 B (one dwordx4)
//   probe_gather32   32 B (two dwordx4 of one line)
//   probe_gather36u  36 B unaligned (nine dwords from a 4 B-aligned base, as load_prefix32)
//   probe_lds_dma1   1 B per lane by global_load_lds_ubyte (the decoder's copy loads)
// usage: traffic_probe [MiB=4096] [accesses=16777216]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                             \
    }                                                                      \
  } while (0)

__global__ void probe_stream16(const uint4 *__restrict__ buf, size_t n16, uint32_t *sink) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) {
    const uint4 v = buf[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}
__global__ void probe_evict(const uint4 *__restrict__ buf, size_t n16, uint32_t *sink) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) {
    const uint4 v = buf[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}
// access i's line: a multiplicative permutation of the line index (odd multiplier, 2^k lines),
// computed in the kernel so the probe reads nothing but the gathered bytes
__device__ __forceinline__ uint64_t line_off(size_t i, uint64_t lmask) { return ((i * 0x9E3779B97F4A7C15ull) & lmask) * 256; }
__global__ void probe_gather1(const uint8_t *__restrict__ buf, uint64_t lmask, size_t n, uint32_t *sink) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) acc += buf[line_off(i, lmask) + 37];
  if (acc == 0x12345678u) sink[0] = acc;
}
__global__ void probe_gather4(const uint8_t *__restrict__ buf, uint64_t lmask, size_t n, uint32_t *sink) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    acc += *(const uint32_t *)(buf + line_off(i, lmask) + 36);
  if (acc == 0x12345678u) sink[0] = acc;
}
__global__ void probe_gather16(const uint8_t *__restrict__ buf, uint64_t lmask, size_t n, uint32_t *sink) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const uint4 v = *(const uint4 *)(buf + line_off(i, lmask) + 32);
    acc += v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}
__global__ void probe_gather32(const uint8_t *__restrict__ buf, uint64_t lmask, size_t n, uint32_t *sink) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const uint4 a = *(const uint4 *)(buf + line_off(i, lmask) + 32), b = *(const uint4 *)(buf + line_off(i, lmask) + 48);
    acc += a.x ^ a.y ^ a.z ^ a.w ^ b.x ^ b.y ^ b.z ^ b.w;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}
__global__ void probe_gather36u(const uint8_t *__restrict__ buf, uint64_t lmask, size_t n, uint32_t *sink) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const uint32_t *w = (const uint32_t *)(buf + line_off(i, lmask) + 100);   // crosses into the next 128 B line
#pragma unroll
    for (int k = 0; k < 9; k++) acc += w[k];
  }
  if (acc == 0x12345678u) sink[0] = acc;
}
__global__ void probe_lds_dma1(const uint8_t *__restrict__ buf, uint64_t lmask, size_t n, uint32_t *sink) {
  __shared__ uint32_t slot[64];
  typedef __attribute__((address_space(3))) void LV;
  typedef __attribute__((address_space(1))) void GV;
  uint32_t acc = 0;
  for (size_t base = blockIdx.x * (size_t)64; base < n; base += (size_t)gridDim.x * 64) {
    const size_t i = base + threadIdx.x;
    const uint8_t *p = buf + (i < n ? line_off(i, lmask) : 0) + 5;
    __builtin_amdgcn_global_load_lds((GV *)p, (LV *)slot, 1, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    acc += slot[threadIdx.x];
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

int main(int argc, char **argv) {
  const size_t mib = argc > 1 ? strtoull(argv[1], 0, 10) : 4096;
  const size_t n = argc > 2 ? strtoull(argv[2], 0, 10) : (16u << 20);
  const size_t bytes = mib << 20, lines = bytes / 256;
  if (n > lines) {
    fprintf(stderr, "more accesses than lines\n");
    return 1;
  }
  uint8_t *buf, *ev;
  uint32_t *sink;
  CK(hipMalloc(&buf, bytes));
  CK(hipMemset(buf, 1, bytes));
  const size_t evb = 1024ull << 20;   // eviction stream: 1 GiB of its own
  CK(hipMalloc(&ev, evb));
  CK(hipMemset(ev, 2, evb));
  CK(hipMalloc(&sink, 4));
  if (lines & (lines - 1)) {
    fprintf(stderr, "MiB must make a power-of-two number of 256 B lines\n");
    return 1;
  }
  const uint64_t lmask = lines - 1;
  const dim3 g(4096), b(256);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto run = [&](const char *name, auto launch, double alg) {
    CK(hipDeviceSynchronize());
    // (evict: stream 1 GiB of another buffer first so no line is in L2 / Infinity Cache)
    hipLaunchKernelGGL(probe_evict, g, b, 0, 0, (const uint4 *)ev, evb / 16, sink);
    CK(hipEventRecord(e0));
    launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("{\"kernel\": \"%s\", \"accesses\": %zu, \"algorithmic_bytes\": %.0f, \"ms\": %.3f}\n", name, n, alg, ms);
  };
  run("probe_stream16", [&] { hipLaunchKernelGGL(probe_stream16, g, b, 0, 0, (const uint4 *)buf, bytes / 2 / 16, sink); },
      (double)(bytes / 2));
  run("probe_gather1", [&] { hipLaunchKernelGGL(probe_gather1, g, b, 0, 0, buf, lmask, n, sink); }, (double)n);
  run("probe_gather4", [&] { hipLaunchKernelGGL(probe_gather4, g, b, 0, 0, buf, lmask, n, sink); }, 4.0 * n);
  run("probe_gather16", [&] { hipLaunchKernelGGL(probe_gather16, g, b, 0, 0, buf, lmask, n, sink); }, 16.0 * n);
  run("probe_gather32", [&] { hipLaunchKernelGGL(probe_gather32, g, b, 0, 0, buf, lmask, n, sink); }, 32.0 * n);
  run("probe_gather36u", [&] { hipLaunchKernelGGL(probe_gather36u, g, b, 0, 0, buf, lmask, n, sink); }, 36.0 * n);
  run("probe_lds_dma1", [&] { hipLaunchKernelGGL(probe_lds_dma1, dim3(8192), dim3(64), 0, 0, buf, lmask, n, sink); }, (double)n);
  CK(hipDeviceSynchronize());
  return 0;
}
