// VALU issue-rate microbenchmark for gfx950 (MI355X).
//
// Measures, for each integer instruction the secp256k1 kernels lean on, the
// sustained wave64-instruction throughput per SIMD, with 16 independent
// dependency chains per wave so latency is hidden. The clock is measured
// in-kernel (s_memtime / s_memrealtime) so the result is in cycles, not ns.
//
// Build: hipcc --offload-arch=gfx950 -O3 -o ubench_valu tools/ubench_valu.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

constexpr int ITERS = 2048;

// Each OP is one asm statement acting on register set i (16 independent sets).
#define REP16(M) M(0) M(1) M(2) M(3) M(4) M(5) M(6) M(7) M(8) M(9) M(10) M(11) M(12) M(13) M(14) M(15)

template <int OP>
__global__ void __launch_bounds__(256) kern(uint32_t* out, uint64_t* clk, uint32_t seed) {
  uint32_t a[16];
  uint64_t w[16];
  double d[16];
  for (int i = 0; i < 16; ++i) {
    a[i] = seed * (threadIdx.x + 7 * i + 1);
    w[i] = (uint64_t)a[i] * 0x9E3779B97F4A7C15ull;
    d[i] = (double)a[i];
  }
  uint32_t b = seed ^ 0x1234567u;
  uint32_t c = seed ^ 0x7654321u;
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  uint64_t r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < ITERS; ++it) {
    if constexpr (OP == 0) {  // v_add_u32
#define M(i) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
      REP16(M)
#undef M
    } else if constexpr (OP == 1) {  // v_mad_u64_u32
#define M(i) { uint64_t cy; asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(w[i]), "=s"(cy) : "v"(b), "v"(c)); }
      REP16(M)
#undef M
    } else if constexpr (OP == 2) {  // v_mul_lo_u32
#define M(i) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
      REP16(M)
#undef M
    } else if constexpr (OP == 3) {  // v_mul_hi_u32
#define M(i) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
      REP16(M)
#undef M
    } else if constexpr (OP == 4) {  // v_mul_u32_u24
#define M(i) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a[i]) : "v"(b));
      REP16(M)
#undef M
    } else if constexpr (OP == 5) {  // v_mul_hi_u32_u24
#define M(i) asm volatile("v_mul_hi_u32_u24 %0, %0, %1" : "+v"(a[i]) : "v"(b));
      REP16(M)
#undef M
    } else if constexpr (OP == 6) {  // v_add_co_u32 (carry out to SGPR pair)
#define M(i) { uint64_t cy; asm volatile("v_add_co_u32 %0, %1, %0, %2" : "+v"(a[i]), "=s"(cy) : "v"(b)); }
      REP16(M)
#undef M
    } else if constexpr (OP == 7) {  // v_addc_co_u32 (carry in/out through VCC chain)
#define M(i) asm volatile("v_addc_co_u32 %0, vcc, %0, %1, vcc" : "+v"(a[i]) : "v"(b) : "vcc");
      REP16(M)
#undef M
    } else if constexpr (OP == 8) {  // v_fma_f64
#define M(i) asm volatile("v_fma_f64 %0, %0, %1, %0" : "+v"(d[i]) : "v"(1.0000001));
      REP16(M)
#undef M
    } else if constexpr (OP == 9) {  // v_mad_u32_u24
#define M(i) asm volatile("v_mad_u32_u24 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));
      REP16(M)
#undef M
    } else if constexpr (OP == 10) {  // v_add3_u32
#define M(i) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));
      REP16(M)
#undef M
    } else if constexpr (OP == 11) {  // v_alignbit_b32 (rotate)
#define M(i) asm volatile("v_alignbit_b32 %0, %0, %1, 7" : "+v"(a[i]) : "v"(b));
      REP16(M)
#undef M
    } else if constexpr (OP == 12) {  // v_cndmask_b32
#define M(i) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a[i]) : "v"(b));
      REP16(M)
#undef M
    } else if constexpr (OP == 13) {  // v_lshl_add_u64 (gfx950 64-bit shift-add)
#define M(i) asm volatile("v_lshl_add_u64 %0, %0, 1, %1" : "+v"(w[i]) : "v"((uint64_t)b));
      REP16(M)
#undef M
    } else if constexpr (OP == 14) {  // v_mad_u64_u32 dependent chain (latency)
      { uint64_t cy; asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(w[0]), "=s"(cy) : "v"(b), "v"(c)); }
    } else if constexpr (OP == 15) {  // v_add_u32 dependent chain (latency)
      asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[0]) : "v"(b));
    } else if constexpr (OP == 16) {  // v_bfi_b32
#define M(i) asm volatile("v_bfi_b32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));
      REP16(M)
#undef M
    } else if constexpr (OP == 17) {  // v_xor3_b32
#define M(i) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(a[i]) : "v"(b), "v"(c));
      REP16(M)
#undef M
    } else if constexpr (OP == 19) {  // v_lshrrev_b64
#define M(i) asm volatile("v_lshrrev_b64 %0, 29, %0" : "+v"(w[i]));
      REP16(M)
#undef M
    } else if constexpr (OP == 20) {  // v_and_b32
#define M(i) asm volatile("v_and_b32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
      REP16(M)
#undef M
    } else if constexpr (OP == 21) {  // v_lshrrev_b32
#define M(i) asm volatile("v_lshrrev_b32 %0, 29, %0" : "+v"(a[i]));
      REP16(M)
#undef M
    } else if constexpr (OP == 22) {  // v_bfe_u32
#define M(i) asm volatile("v_bfe_u32 %0, %0, 3, 29" : "+v"(a[i]));
      REP16(M)
#undef M
    } else if constexpr (OP == 23) {  // v_mov_b32
#define M(i) asm volatile("v_mov_b32 %0, %1" : "=v"(a[i]) : "v"(a[(i + 1) & 15]));
      REP16(M)
#undef M
    } else if constexpr (OP == 24) {  // v_cndmask_b32 with an SGPR-pair mask that no VALU writes
      uint64_t msk = 0x5555555555555555ull ^ b;
      asm volatile("s_mov_b64 %0, %0" : "+s"(msk));
#define M(i) asm volatile("v_cndmask_b32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "s"(msk));
      REP16(M)
#undef M
    } else if constexpr (OP == 25) {  // carry step as compiled: and + 64-bit shift + 64-bit add
#define M(i) asm volatile("v_and_b32 %1, 0x1fffffff, %1\n\tv_lshrrev_b64 %0, 29, %0\n\tv_lshl_add_u64 %0, %0, 0, %2" : "+v"(w[i]), "+v"(a[i]) : "v"(w[(i + 1) & 15]));
      REP16(M)
#undef M
    } else if constexpr (OP == 26) {  // v_lshlrev_b64
#define M(i) asm volatile("v_lshlrev_b64 %0, 3, %0" : "+v"(w[i]));
      REP16(M)
#undef M
    } else if constexpr (OP == 27) {  // v_sub_co_u32 + v_subb_co_u32 (64-bit subtract)
#define M(i) asm volatile("v_sub_co_u32 %0, vcc, %0, %1\n\tv_subb_co_u32 %2, vcc, %2, %1, vcc" : "+v"(a[i]), "+v"(b), "+v"(c) :: "vcc");
      REP16(M)
#undef M
    } else if constexpr (OP == 18) {  // v_pk_mad? -> v_mad_u64_u32 interleaved 1:2 with v_add_u32
#define M(i) { uint64_t cy; asm volatile("v_mad_u64_u32 %0, %2, %3, %4, %0\n\tv_add_u32 %1, %1, %3\n\tv_add_u32 %1, %1, %4" : "+v"(w[i]), "+v"(a[i]), "=s"(cy) : "v"(b), "v"(c)); }
      REP16(M)
#undef M
    }
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  uint64_t r1 = __builtin_amdgcn_s_memrealtime();
  uint32_t acc = 0;
  for (int i = 0; i < 16; ++i) acc += a[i] + (uint32_t)w[i] + (uint32_t)(w[i] >> 32) + (uint32_t)d[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = t1 - t0; clk[1] = r1 - r0; }
}

template <int OP>
void run(const char* name, int insts_per_stmt, int chains, int blocks_per_cu) {
  int ncu = 256;
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  ncu = prop.multiProcessorCount;
  int blocks = ncu * blocks_per_cu;
  uint32_t* out; uint64_t* clk;
  CHECK(hipMalloc(&out, (size_t)blocks * 256 * 4));
  CHECK(hipMalloc(&clk, 16));
  hipLaunchKernelGGL(kern<OP>, dim3(blocks), dim3(256), 0, 0, out, clk, 3u);
  CHECK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  CHECK(hipEventRecord(e0));
  const int reps = 5;
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(kern<OP>, dim3(blocks), dim3(256), 0, 0, out, clk, 3u + r);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
  uint64_t hclk[2]; CHECK(hipMemcpy(hclk, clk, 16, hipMemcpyDeviceToHost));
  double ghz = (double)hclk[0] / ((double)hclk[1] / 100e6) / 1e9;  // memrealtime is 100 MHz
  double waves = (double)blocks * 4.0 * reps;
  double inst = waves * ITERS * chains * insts_per_stmt;  // wave-instructions
  double sec = ms / 1e3;
  // cycles per wave-instruction per SIMD (4 SIMDs per CU), at the in-kernel clock
  double simd_cycles = sec * ghz * 1e9 * ncu * 4;
  double cpi = simd_cycles / inst;
  double lane_ops = inst * 64 / sec;
  printf("%-22s %8.3f ms  clk %.2f GHz  %6.2f cyc/wave-inst/SIMD  %8.2f Tlane-op/s\n", name, ms / reps, ghz, cpi,
         lane_ops / 1e12);
  CHECK(hipFree(out)); CHECK(hipFree(clk));
}

int main() {
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  printf("device %s  CUs %d  clock %d kHz\n", prop.gcnArchName, prop.multiProcessorCount, prop.clockRate);
  for (int bpc = 2; bpc <= 4; bpc += 2) {
    printf("--- %d blocks of 256 per CU (%d waves/SIMD) ---\n", bpc, bpc);
    run<0>("v_add_u32", 1, 16, bpc);
    run<1>("v_mad_u64_u32", 1, 16, bpc);
    run<2>("v_mul_lo_u32", 1, 16, bpc);
    run<3>("v_mul_hi_u32", 1, 16, bpc);
    run<4>("v_mul_u32_u24", 1, 16, bpc);
    run<5>("v_mul_hi_u32_u24", 1, 16, bpc);
    run<6>("v_add_co_u32", 1, 16, bpc);
    run<7>("v_addc_co_u32(vcc)", 1, 16, bpc);
    run<8>("v_fma_f64", 1, 16, bpc);
    run<9>("v_mad_u32_u24", 1, 16, bpc);
    run<10>("v_add3_u32", 1, 16, bpc);
    run<11>("v_alignbit_b32", 1, 16, bpc);
    run<12>("v_cndmask_b32", 1, 16, bpc);
    run<13>("v_lshl_add_u64", 1, 16, bpc);
    run<16>("v_bfi_b32", 1, 16, bpc);
    run<17>("v_bitop3_b32(xor3)", 1, 16, bpc);
    run<18>("mad64+2add mix", 3, 16, bpc);
    run<19>("v_lshrrev_b64", 1, 16, bpc);
    run<26>("v_lshlrev_b64", 1, 16, bpc);
    run<20>("v_and_b32", 1, 16, bpc);
    run<21>("v_lshrrev_b32", 1, 16, bpc);
    run<22>("v_bfe_u32", 1, 16, bpc);
    run<23>("v_mov_b32", 1, 16, bpc);
    run<24>("v_cndmask_b32(sgpr)", 1, 16, bpc);
    run<25>("carry step (3 ops)", 3, 16, bpc);
    run<27>("sub_co+subb_co", 2, 16, bpc);
  }
  printf("--- latency (1 chain, 1 wave/SIMD) ---\n");
  run<14>("v_mad_u64_u32 dep", 1, 1, 1);
  run<15>("v_add_u32 dep", 1, 1, 1);
  return 0;
}
