// probe: where does global_load_lds_ubyte put lane l's byte in LDS (stride 1 or 4)?
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef __attribute__((address_space(3))) void LV;
typedef __attribute__((address_space(1))) void GV;
__global__ void probe(const unsigned char *src, unsigned char *out) {
  __shared__ unsigned char buf[512];
  for (int i = threadIdx.x; i < 512; i += 64) buf[i] = 0xEE;
  __syncthreads();
  __builtin_amdgcn_global_load_lds((GV *)(src + threadIdx.x), (LV *)buf, 1, 0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int i = threadIdx.x; i < 512; i += 64) out[i] = buf[i];
}
int main() {
  unsigned char h[64], *d, *o, r[512];
  for (int i = 0; i < 64; i++) h[i] = (unsigned char)(i + 1);
  hipMalloc(&d, 64); hipMalloc(&o, 512);
  hipMemcpy(d, h, 64, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d, o);
  hipMemcpy(r, o, 512, hipMemcpyDeviceToHost);
  for (int i = 0; i < 272; i++) printf("%02x%s", r[i], (i % 32 == 31) ? "\n" : " ");
  printf("\n");
  return 0;
}
