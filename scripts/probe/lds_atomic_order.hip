// Probe (MI355X): for one wave's ds_add_rtn_u32 with colliding addresses, are the returned
// values ascending in lane order per address?  (The bucket sort's stable ranking would use it.)
// Prints the number of trials and violations.
#include <hip/hip_runtime.h>
#include <stdio.h>
__global__ void probe(const unsigned *addr, int trials, unsigned *bad) {
  __shared__ unsigned cnt[64][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  unsigned nbad = 0;
  for (int t = blockIdx.x * 4 + w; t < trials; t += gridDim.x * 4) {
    for (int i = 0; i < 64; i++) cnt[w][i] = 0;
    __builtin_amdgcn_wave_barrier();
    const unsigned a = addr[t * 64 + lane];
    const unsigned r = atomicAdd(&cnt[w][a], 1u);
    __builtin_amdgcn_wave_barrier();
    // rank among lower lanes with the same address
    unsigned below = 0;
    for (int l = 0; l < 64; l++) {
      const unsigned al = __shfl(a, l);
      below += (l < lane && al == a) ? 1u : 0u;
    }
    nbad += r != below ? 1u : 0u;
  }
  atomicAdd(bad, nbad);
}
int main() {
  const int trials = 1 << 16;
  unsigned *h = (unsigned *)malloc(sizeof(unsigned) * trials * 64);
  unsigned x = 12345;
  for (int t = 0; t < trials; t++) {
    const unsigned range = 1 + (t % 64);   // 1..64 distinct addresses
    for (int l = 0; l < 64; l++) {
      x ^= x << 13; x ^= x >> 17; x ^= x << 5;
      h[t * 64 + l] = x % range;
    }
  }
  unsigned *d, *bad;
  hipMalloc(&d, sizeof(unsigned) * trials * 64);
  hipMalloc(&bad, 4);
  hipMemcpy(d, h, sizeof(unsigned) * trials * 64, hipMemcpyHostToDevice);
  hipMemset(bad, 0, 4);
  hipLaunchKernelGGL(probe, dim3(256), dim3(256), 0, 0, d, trials, bad);
  unsigned nb = 0;
  hipMemcpy(&nb, bad, 4, hipMemcpyDeviceToHost);
  printf("trials %d lanes with a rank other than their lane order: %u\n", trials, nb);
  return 0;
}
