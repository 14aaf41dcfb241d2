// Where the waves of a 5-wave workgroup land (one workgroup per CU: 100 KB of LDS each): for
// each wave index, the SIMD (HW_ID bits 5:4) it ran on, over 256 workgroups. Build:
// hipcc --offload-arch=gfx950 -O2 -o tools/place_probe tools/place_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

__global__ void __launch_bounds__(320, 1) probe(unsigned* out) {
  extern __shared__ unsigned lds[];
  const unsigned w = threadIdx.x >> 6;
  unsigned hw;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
  lds[threadIdx.x] = hw;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) out[blockIdx.x * 5 + w] = hw;
}

int main() {
  const int blocks = 256;
  unsigned* d;
  if (hipMalloc(&d, blocks * 5 * sizeof(unsigned)) != hipSuccess) return 1;
  hipLaunchKernelGGL(probe, dim3(blocks), dim3(320), 100 * 1024, 0, d);
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  std::vector<unsigned> h(blocks * 5);
  if (hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost) != hipSuccess) return 3;
  int cnt[5][4] = {};
  int same04 = 0, same14 = 0;
  for (int b = 0; b < blocks; ++b) {
    for (int w = 0; w < 5; ++w) cnt[w][(h[b * 5 + w] >> 4) & 3]++;
    const unsigned s0 = (h[b * 5] >> 4) & 3, s1 = (h[b * 5 + 1] >> 4) & 3, s4 = (h[b * 5 + 4] >> 4) & 3;
    same04 += s0 == s4;
    same14 += s1 == s4;
  }
  for (int w = 0; w < 5; ++w) printf("wave %d SIMD counts: %d %d %d %d\n", w, cnt[w][0], cnt[w][1], cnt[w][2], cnt[w][3]);
  printf("wave 4 on wave 0's SIMD: %d / %d, on wave 1's SIMD: %d / %d\n", same04, blocks, same14, blocks);
  return 0;
}
