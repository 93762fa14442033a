// Probe (MI355X): cycles per step of the dependent chains a literal decode is built from, one
// wave alone and one wave per SIMD (1024 waves):
//   lds_s   : uniform LDS u16 load -> readfirstlane -> scalar math -> next address
//   lds_v   : the same chain kept in VGPRs (no readfirstlane)
//   rlane   : v_readlane with an SGPR lane select -> scalar math -> next select
//   bperm   : ds_bpermute chain
//   spec    : 64-lane speculative lookup (lane l at offset x + l) + readlane walk of 8 steps
// Prints s_memtime ticks per step.
#include <hip/hip_runtime.h>
#include <stdio.h>
__shared__ uint16_t tab[16384];
__global__ __launch_bounds__(64) void chain(int mode, int iters, unsigned long long *cyc, int *sink) {
  const int lane = threadIdx.x;
  for (int i = lane; i < 16384; i += 64) tab[i] = (uint16_t)((i * 2654435761u >> 7) & 0x3FFF);
  __syncthreads();
  uint32_t x = blockIdx.x & 255, vx = x, acc = 0;
  const uint32_t lv = (lane * 40503u) & 0x3FFF;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  if (mode == 0) {
    for (int i = 0; i < iters; i++) {
      const uint32_t e = (uint32_t)__builtin_amdgcn_readfirstlane((int)tab[x]);
      x = ((e >> 3) ^ i) & 0x3FFF;
    }
  } else if (mode == 1) {
    for (int i = 0; i < iters; i++) {
      const uint32_t e = tab[vx];
      vx = ((e >> 3) ^ (uint32_t)i) & 0x3FFF;
    }
    x = (uint32_t)__builtin_amdgcn_readfirstlane((int)vx);
  } else if (mode == 2) {
    for (int i = 0; i < iters; i++) {
      const uint32_t e = (uint32_t)__builtin_amdgcn_readlane((int)lv, (int)(x & 63));
      x = (e >> 3) ^ (uint32_t)i;
    }
  } else if (mode == 3) {
    for (int i = 0; i < iters; i++) {
      const uint32_t e = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((vx & 63) << 2), (int)lv);
      vx = (e >> 3) ^ (uint32_t)i;
    }
    x = (uint32_t)__builtin_amdgcn_readfirstlane((int)vx);
  } else {
    // one LDS round trip per 8 readlane steps
    for (int i = 0; i < iters; i += 8) {
      const uint32_t e = tab[(x + lane) & 0x3FFF];
      uint32_t o = 0;
#pragma unroll
      for (int k = 0; k < 8; k++) {
        const uint32_t v = (uint32_t)__builtin_amdgcn_readlane((int)e, (int)(o & 63));
        o += 1 + (v & 3);
        acc += v;
      }
      x = (x + o) & 0x3FFF;
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) {
    atomicAdd(cyc, t1 - t0);
    sink[blockIdx.x] = (int)(x + acc);
  }
}
int main() {
  unsigned long long *cyc, h;
  int *sink;
  hipMalloc(&cyc, 8);
  hipMalloc(&sink, 4096 * 4);
  const char *names[5] = {"lds_s", "lds_v", "rlane", "bperm", "spec8"};
  const int iters = 8000;
  for (int m = 0; m < 5; m++) {
    for (int waves : {1, 1024}) {
      double r = 0;
      for (int rep = 0; rep < 2; rep++) {
        hipMemset(cyc, 0, 8);
        hipLaunchKernelGGL(chain, dim3(waves), dim3(64), 0, 0, m, iters, cyc, sink);
        hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost);
        r = (double)h / waves / iters;
      }
      printf("%-6s %5d waves: %.1f ticks per step\n", names[m], waves, r);
    }
  }
  // the tick rate: one wave, mode 0, timed by events
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipMemset(cyc, 0, 8);
  hipEventRecord(a, 0);
  hipLaunchKernelGGL(chain, dim3(1), dim3(64), 0, 0, 0, 400000, cyc, sink);
  hipEventRecord(b, 0);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost);
  printf("tick rate: %.1f MHz (%llu ticks in %.3f ms)\n", (double)h / ms / 1e3, h, ms);
  return 0;
}
