// Probe (MI355X): the latency a decoder wave sees for a copy source, i.e. a dependent byte
// load 8 KiB..1 MiB back in the wave's own recently written 1 MiB region, with 1024 waves
// (one per SIMD) doing the same.  Variants: plain global load vs LDS-DMA; with / without the
// decoder's stream of output stores.  Prints cycles per dependent load (s_memtime).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
__shared__ uint32_t slot[64];
template <bool kDma, bool kStores>
__global__ __launch_bounds__(64) void chase(uint8_t *buf, int iters, unsigned long long *cyc) {
  uint8_t *base = buf + ((size_t)blockIdx.x << 20);
  const int lane = threadIdx.x;
  uint32_t x = 0x9E3779B9u * (blockIdx.x + 1);
  int pos = 1 << 19;
  uint32_t acc = 0;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; i++) {
    x ^= x << 13; x ^= x >> 17; x ^= x << 5;
    x += acc;   // dependent on the previous load
    const int dist = 8192 + (int)(x % (512u << 10));
    const int src = (pos - dist) & ((1 << 20) - 1);
    uint32_t v;
    if (kDma) {
      typedef __attribute__((address_space(3))) void LV;
      typedef __attribute__((address_space(1))) void GV;
      __builtin_amdgcn_global_load_lds((GV *)(base + ((src + lane) & ((1 << 20) - 1))), (LV *)slot, 1, 0, 0);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      v = slot[lane];
    } else {
      v = base[(src + lane) & ((1 << 20) - 1)];
    }
    acc = __builtin_amdgcn_readfirstlane((int)v);
    if (kStores) {   // ~10 output bytes per command
      if (lane < 10) base[(pos + lane) & ((1 << 20) - 1)] = (uint8_t)(v + i);
      pos = (pos + 10) & ((1 << 20) - 1);
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) atomicAdd(cyc, t1 - t0 + (acc == 12345 ? 1 : 0));
}
int main() {
  const int waves = 1024, iters = 4000;
  uint8_t *buf;
  unsigned long long *cyc, h;
  hipMalloc(&buf, (size_t)waves << 20);
  hipMemset(buf, 1, (size_t)waves << 20);
  hipMalloc(&cyc, 8);
  const char *names[4] = {"load", "load+stores", "dma", "dma+stores"};
  for (int v = 0; v < 4; v++) {
    for (int rep = 0; rep < 2; rep++) {
      hipMemset(cyc, 0, 8);
      if (v == 0) hipLaunchKernelGGL((chase<false, false>), dim3(waves), dim3(64), 0, 0, buf, iters, cyc);
      if (v == 1) hipLaunchKernelGGL((chase<false, true>), dim3(waves), dim3(64), 0, 0, buf, iters, cyc);
      if (v == 2) hipLaunchKernelGGL((chase<true, false>), dim3(waves), dim3(64), 0, 0, buf, iters, cyc);
      if (v == 3) hipLaunchKernelGGL((chase<true, true>), dim3(waves), dim3(64), 0, 0, buf, iters, cyc);
      hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost);
      if (rep) printf("%-12s %.0f cycles per dependent load (1024 waves)\n", names[v], (double)h / waves / iters);
    }
  }
  // one wave alone
  hipMemset(cyc, 0, 8);
  hipLaunchKernelGGL((chase<true, true>), dim3(1), dim3(64), 0, 0, buf, iters, cyc);
  hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost);
  printf("%-12s %.0f cycles per dependent load (1 wave)\n", "dma+stores", (double)h / iters);
  return 0;
}
