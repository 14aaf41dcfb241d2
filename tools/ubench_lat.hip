// Single-wave latency microbenchmark for gfx950 (MI355X): what one dependent instruction costs a
// wave that has its SIMD to itself (the latency kernels' situation: one signature's chain per
// wave). One workgroup of one wave; s_memtime (shader clock) around a loop of
// UNROLL dependent instructions per iteration.
//
// Build: hipcc --offload-arch=gfx950 -O3 -o ubench_lat tools/ubench_lat.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                                 \
  do {                                                                                           \
    hipError_t e_ = (x);                                                                         \
    if (e_ != hipSuccess) {                                                                      \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__);    \
      exit(1);                                                                                   \
    }                                                                                            \
  } while (0)

constexpr int ITERS = 512;
#define R8(S) S S S S S S S S

template <int OP>
__global__ void __launch_bounds__(64) kern(uint32_t* out, uint64_t* clk, uint32_t seed) {
  __shared__ uint32_t lds[256];
  for (int i = threadIdx.x; i < 256; i += 64) lds[i] = (uint32_t)(i + 1) & 255u;  // chase: i -> i + 1
  __syncthreads();
  uint32_t s0 = seed, s1 = seed * 3u + 1u;
  uint64_t s64 = ((uint64_t)seed << 32) | 0x9E3779B9u;
  uint32_t v0 = seed + threadIdx.x, v1 = seed ^ threadIdx.x, v2 = 7u * threadIdx.x + 1u;
  uint64_t v64 = ((uint64_t)v0 << 32) | v1, w1 = v64 * 3u, w2 = v64 * 5u, w3 = v64 * 7u;
  asm volatile("" : "+s"(s0), "+s"(s1), "+s"(s64), "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v64), "+v"(w1), "+v"(w2), "+v"(w3));
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
  for (int it = 0; it < ITERS; ++it) {
    if constexpr (OP == 0) {
      R8(asm volatile("s_add_u32 %0, %0, %1" : "+s"(s0) : "s"(s1));)
    } else if constexpr (OP == 1) {
      R8(asm volatile("s_mul_i32 %0, %0, %1" : "+s"(s0) : "s"(s1));)
    } else if constexpr (OP == 2) {
      R8(asm volatile("s_lshr_b64 %0, %0, 1" : "+s"(s64));)
    } else if constexpr (OP == 3) {  // 64-bit add: 2 instructions
      R8(asm volatile("s_add_u32 %0, %0, %2\n s_addc_u32 %1, %1, 0" : "+s"(s0), "+s"(s1) : "s"(seed) : "scc");)
    } else if constexpr (OP == 4) {  // ctz + shift: 2 instructions
      R8(asm volatile("s_ff1_i32_b32 %1, %0\n s_lshr_b32 %0, %0, %1" : "+s"(s0), "=&s"(s1) : : "scc");)
    } else if constexpr (OP == 5) {  // compare + select: 2 instructions
      R8(asm volatile("s_cmp_lt_u32 %0, %1\n s_cselect_b32 %0, %1, %0" : "+s"(s0) : "s"(s1) : "scc");)
    } else if constexpr (OP == 6) {
      R8(asm volatile("v_add_u32 %0, %0, %1" : "+v"(v0) : "v"(v1));)
    } else if constexpr (OP == 7) {
      R8({ uint64_t cy; asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(v64), "=s"(cy) : "v"(v1), "v"(v2)); })
    } else if constexpr (OP == 8) {  // VALU -> SALU -> VALU round trip: 3 instructions
      R8(asm volatile("v_readfirstlane_b32 %1, %0\n s_add_u32 %1, %1, 1\n v_mov_b32 %0, %1" : "+v"(v0), "=&s"(s1) : : "scc");)
    } else if constexpr (OP == 9) {  // DPP row shift
      R8(asm volatile("v_add_u32_dpp %0, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(v0));)
    } else if constexpr (OP == 10) {  // ds_bpermute (address from the value): 2 instructions + wait
      R8(asm volatile("v_and_b32 %1, 0xfc, %0\n ds_bpermute_b32 %0, %1, %0\n s_waitcnt lgkmcnt(0)" : "+v"(v0), "=&v"(v2));)
    } else if constexpr (OP == 11) {  // LDS pointer chase: ds_read + wait (+ shift)
      R8(asm volatile("v_lshlrev_b32 %0, 2, %0\n ds_read_b32 %0, %0\n s_waitcnt lgkmcnt(0)" : "+v"(v0));)
    } else if constexpr (OP == 12) {
      R8(asm volatile("v_lshlrev_b64 %0, 1, %0" : "+v"(v64));)
    } else if constexpr (OP == 13) {
      R8(asm volatile("s_min_i32 %0, %0, %1" : "+s"(s0) : "s"(s1));)
    } else if constexpr (OP == 14) {  // two independent SALU chains interleaved: 2 instructions
      R8(asm volatile("s_add_u32 %0, %0, 3\n s_add_u32 %1, %1, 5" : "+s"(s0), "+s"(s1) : : "scc");)
    } else if constexpr (OP == 15) {  // two independent VALU chains interleaved: 2 instructions
      R8(asm volatile("v_add_u32 %0, %0, %2\n v_add_u32 %1, %1, %2" : "+v"(v0), "+v"(v1) : "v"(v2));)
    } else if constexpr (OP == 16) {  // independent VALU and SALU chains interleaved: 2 instructions
      R8(asm volatile("v_add_u32 %0, %0, %2\n s_add_u32 %1, %1, 5" : "+v"(v0), "+s"(s1) : "v"(v2) : "scc");)
    } else if constexpr (OP == 17) {  // four independent v_mad_u64 chains: 4 instructions
      R8({
        uint64_t cy;
        asm volatile("v_mad_u64_u32 %0, %1, %6, %7, %0\n v_mad_u64_u32 %2, %1, %6, %7, %2\n"
                     " v_mad_u64_u32 %3, %1, %6, %7, %3\n v_mad_u64_u32 %4, %1, %6, %7, %4"
                     : "+v"(v64), "=s"(cy), "+v"(w1), "+v"(w2), "+v"(w3) : "v"(v0), "v"(v1), "v"(v2));
      })
    } else if constexpr (OP == 18) {  // s_mul_hi_u32
      R8(asm volatile("s_mul_hi_u32 %0, %0, %1" : "+s"(s0) : "s"(s1));)
    } else if constexpr (OP == 19) {  // v_mul_lo_u32 dependent
      R8(asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(v0) : "v"(v1));)
    } else if constexpr (OP == 20) {  // v_permlane32_swap
      R8({ const auto p_ = __builtin_amdgcn_permlane32_swap(v0, v0, false, false); v0 = p_[0] + p_[1]; asm volatile("" : "+v"(v0)); })
    } else if constexpr (OP == 21) {  // s_bcnt1 / s_flbit style op
      R8(asm volatile("s_flbit_i32_b32 %0, %0" : "+s"(s0));)
    }
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = s0 + s1 + (uint32_t)s64 + (uint32_t)(s64 >> 32) + v0 + v1 + v2 + (uint32_t)v64 + (uint32_t)(v64 >> 32) + (uint32_t)(w1 ^ w2 ^ w3);
  if (threadIdx.x == 0) clk[0] = t1 - t0;
}

template <int OP>
void run(const char* name, int insts_per_stmt) {
  uint32_t* out;
  uint64_t* clk;
  CHECK(hipMalloc(&out, 64 * 4));
  CHECK(hipMalloc(&clk, 8));
  double best = 1e30;
  for (int r = 0; r < 5; ++r) {
    hipLaunchKernelGGL(kern<OP>, dim3(1), dim3(64), 0, 0, out, clk, 3u + r);
    CHECK(hipDeviceSynchronize());
    uint64_t c;
    CHECK(hipMemcpy(&c, clk, 8, hipMemcpyDeviceToHost));
    const double per = (double)c / ((double)ITERS * 8 * insts_per_stmt);
    if (per < best) best = per;
  }
  printf("%-34s %7.2f cycles per instruction (%d per statement)\n", name, best, insts_per_stmt);
  CHECK(hipFree(out));
  CHECK(hipFree(clk));
}

int main() {
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  printf("device %s  one wave, dependent chains, s_memtime cycles (loop overhead included)\n", prop.gcnArchName);
  run<0>("s_add_u32 dep", 1);
  run<13>("s_min_i32 dep", 1);
  run<1>("s_mul_i32 dep", 1);
  run<18>("s_mul_hi_u32 dep", 1);
  run<2>("s_lshr_b64 dep", 1);
  run<3>("s_add_u32+s_addc_u32 dep", 2);
  run<4>("s_ff1+s_lshr dep", 2);
  run<5>("s_cmp+s_cselect dep", 2);
  run<21>("s_flbit dep", 1);
  run<14>("2 indep SALU chains", 2);
  run<6>("v_add_u32 dep", 1);
  run<15>("2 indep v_add chains", 2);
  run<16>("v_add + s_add indep", 2);
  run<7>("v_mad_u64_u32 dep", 1);
  run<17>("4 indep v_mad_u64 chains", 4);
  run<19>("v_mul_lo_u32 dep", 1);
  run<12>("v_lshlrev_b64 dep", 1);
  run<9>("v_add_dpp row_shr dep", 1);
  run<20>("permlane32_swap+v_add dep", 2);
  run<8>("readfirstlane+s_add+v_mov dep", 3);
  run<10>("v_and+ds_bpermute+wait dep", 3);
  run<11>("v_lshl+ds_read+wait dep", 3);
  return 0;
}
