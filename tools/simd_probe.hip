#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
__global__ void __launch_bounds__(256, 2) probe(uint32_t* out, int spin) {
  __shared__ uint32_t big[19000];  // ~76 KB: two workgroups per CU
  uint32_t hw, xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  big[threadIdx.x] = hw;
  __syncthreads();
  uint64_t t = t0;
  while (t - t0 < (uint64_t)spin) t = __builtin_amdgcn_s_memrealtime();
  const int w = threadIdx.x / 64;
  if ((threadIdx.x & 63) == 0) {
    uint32_t* o = out + 4 * (blockIdx.x * 4 + w);
    o[0] = hw; o[1] = xcc; o[2] = (uint32_t)t0; o[3] = big[(threadIdx.x + 64) & 255];
  }
}
int main(int argc, char** argv) {
  int nb = argc > 1 ? atoi(argv[1]) : 512;
  uint32_t* d; hipMalloc(&d, nb * 16 * 4);
  probe<<<nb, 256>>>(d, 5000);  // warm
  hipDeviceSynchronize();
  probe<<<nb, 256>>>(d, 5000);  // 50 us spin
  hipDeviceSynchronize();
  uint32_t* h = (uint32_t*)malloc(nb * 16 * 4);
  hipMemcpy(h, d, nb * 16 * 4, hipMemcpyDeviceToHost);
  for (int b = 0; b < nb; ++b)
    for (int w = 0; w < 4; ++w) {
      const uint32_t* o = h + 4 * (b * 4 + w);
      printf("%d %d %u %u %u\n", b, w, o[0], o[1], o[2]);
    }
  return 0;
}
