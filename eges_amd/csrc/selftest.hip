// Field / group self-test kernels (test harness only: libeges_selftest.so, used by
// tests/test_gpu_field.py; not part of libeges.so). Inputs and outputs are canonical 256-bit
// integers as 8 little-endian 32-bit words; the Python side checks against big integers.
#include <hip/hip_runtime.h>

#include <vector>

#include "core.cuh"

namespace eges {

// op codes
enum : int {
  OP_MUL = 0,      // a * b
  OP_SQR = 1,      // a^2
  OP_ADD = 2,      // a + b
  OP_SUB = 3,      // a - b
  OP_INV = 4,      // a^-1
  OP_SQRT = 5,     // sqrt(a) (out) and is-square flag (flag)
  OP_LAZY = 6,     // (2a) * (a + 2b) - 2b*(a - b) with maximal lazy magnitudes (2 x 3)
  OP_NEG = 7,      // -a
  OP_EQZ = 8,      // flag = (a == b mod p) via fe_equal on a raw (non-reduced) input
  OP_DBL = 9,      // Jacobian doubling of affine (a, b): out affine x, out2 affine y
  OP_MADD = 10,    // (a,b) + (c,d) affine inputs via Jacobian (Z=1) mixed add; flags h0/r0
  OP_SCMUL = 11,   // a * b mod n
  OP_SCINV = 12,   // a^-1 mod n
  OP_GLV = 13,     // glv split of a: out = |k1|, out2 = |k2| (160-bit), flag = signs
};

__device__ fe ld(const uint32_t* p, uint32_t i) {
  uint32_t x[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) x[k] = p[(size_t)i * 8 + k];
  return fe_from_u256(x);
}
__device__ void st(uint32_t* p, uint32_t i, const fe& a) {
  uint32_t x[8];
  fe_to_u256(x, fe_normalize(a));
#pragma unroll
  for (int k = 0; k < 8; ++k) p[(size_t)i * 8 + k] = x[k];
}

__global__ void selftest_kernel(int op, uint32_t n, const uint32_t* A, const uint32_t* B, const uint32_t* C,
                                const uint32_t* D, uint32_t* out, uint32_t* out2, uint32_t* flag) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const fe a = ld(A, i), b = ld(B, i);
  switch (op) {
    case OP_MUL: st(out, i, fe_mul(a, b)); break;
    case OP_SQR: st(out, i, fe_sqr(a)); break;
    case OP_ADD: st(out, i, fe_add(a, b)); break;
    case OP_SUB: st(out, i, fe_sub<1>(a, b)); break;
    case OP_INV: st(out, i, fe_inv(a)); break;
    case OP_SQRT: {
      fe r;
      const bool ok = fe_sqrt(r, a);
      st(out, i, r);
      flag[i] = ok;
      break;
    }
    case OP_LAZY: {
      const fe a2 = fe_add(a, a);                               // 2
      const fe t = fe_add(a, fe_add(b, b));                     // 3
      const fe u = fe_mul(a2, t);                               // 2 x 3 -> 1
      const fe w = fe_mul(fe_add(b, b), fe_sub<1>(a, b));       // 2 x 3
      st(out, i, fe_sub<1>(u, w));
      break;
    }
    case OP_NEG: st(out, i, fe_neg<1>(a)); break;
    case OP_EQZ: {
      // raw limbs of A taken as a weak value (may be >= p); equality with b
      flag[i] = fe_equal(a, b) ? 1u : 0u;
      break;
    }
    case OP_DBL: {
      gej j;
      j.x = a;
      j.y = b;
      j.z = fe_one();
      gej r = gej_double(gej_double(j));  // 4P, exercises Z != 1
      const fe zi = fe_inv(r.z);
      const fe zi2 = fe_sqr(zi);
      st(out, i, fe_mul(r.x, zi2));
      st(out2, i, fe_mul(r.y, fe_mul(zi2, zi)));
      break;
    }
    case OP_MADD: {
      gej j;
      j.x = a;
      j.y = b;
      j.z = fe_one();
      j = gej_double(j);  // 2P (Z != 1)
      ge q;
      q.x = ld(C, i);
      q.y = ld(D, i);
      bool hz, rz;
      gej r = gej_add_ge(j, q, hz, rz);
      const fe zi = fe_inv(r.z);
      const fe zi2 = fe_sqr(zi);
      st(out, i, fe_mul(r.x, zi2));
      st(out2, i, fe_mul(r.y, fe_mul(zi2, zi)));
      flag[i] = (hz ? 1u : 0u) | (rz ? 2u : 0u);
      break;
    }
    case OP_SCMUL:
    case OP_SCINV: {
      uint32_t x[8], y[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) { x[k] = A[(size_t)i * 8 + k]; y[k] = B[(size_t)i * 8 + k]; }
      bool o1, o2;
      sc s1 = sc_from_limbs(x, o1), s2 = sc_from_limbs(y, o2);
      sc r = op == OP_SCMUL ? sc_mul(s1, s2) : sc_inv(s1);
#pragma unroll
      for (int k = 0; k < 8; ++k) out[(size_t)i * 8 + k] = r.v[k];
      break;
    }
    case OP_GLV: {
      uint32_t x[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) x[k] = A[(size_t)i * 8 + k];
      bool o;
      sc s = sc_from_limbs(x, o);
      glv_half h1, h2;
      glv_split(h1, h2, s);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        out[(size_t)i * 8 + k] = k < 5 ? h1.mag[k] : 0u;
        out2[(size_t)i * 8 + k] = k < 5 ? h2.mag[k] : 0u;
      }
      flag[i] = (h1.neg ? 1u : 0u) | (h2.neg ? 2u : 0u);
      break;
    }
  }
}

}  // namespace eges

extern "C" int eges_selftest(int op, uint32_t n, const uint32_t* a, const uint32_t* b, const uint32_t* c,
                             const uint32_t* d, uint32_t* out, uint32_t* out2, uint32_t* flag) {
  const size_t B = (size_t)n * 32;
  uint32_t *da, *db, *dc, *dd, *dout, *dout2, *dflag;
  if (hipMalloc(&da, B) || hipMalloc(&db, B) || hipMalloc(&dc, B) || hipMalloc(&dd, B) || hipMalloc(&dout, B) ||
      hipMalloc(&dout2, B) || hipMalloc(&dflag, (size_t)n * 4))
    return -1;
  (void)hipMemcpy(da, a, B, hipMemcpyHostToDevice);
  (void)hipMemcpy(db, b, B, hipMemcpyHostToDevice);
  (void)hipMemcpy(dc, c, B, hipMemcpyHostToDevice);
  (void)hipMemcpy(dd, d, B, hipMemcpyHostToDevice);
  (void)hipMemset(dflag, 0, (size_t)n * 4);
  hipLaunchKernelGGL(eges::selftest_kernel, dim3((n + 127) / 128), dim3(128), 0, 0, op, n, da, db, dc, dd, dout, dout2,
                     dflag);
  hipError_t e = hipDeviceSynchronize();
  (void)hipMemcpy(out, dout, B, hipMemcpyDeviceToHost);
  (void)hipMemcpy(out2, dout2, B, hipMemcpyDeviceToHost);
  (void)hipMemcpy(flag, dflag, (size_t)n * 4, hipMemcpyDeviceToHost);
  (void)hipFree(da); (void)hipFree(db); (void)hipFree(dc); (void)hipFree(dd); (void)hipFree(dout); (void)hipFree(dout2); (void)hipFree(dflag);
  return e == hipSuccess ? 0 : -2;
}

// ---------------------------------------------------------------- ecmult_core
// Q = ur * P + ug * G through the kernels' Strauss core (fast path + exact redo), affine out;
// flag = 1 when Q is infinity. Exercises the exceptional-sum handling with chosen scalars.
namespace eges {
__global__ void __launch_bounds__(WG) selftest_ecmult_kernel(uint32_t n, const uint32_t* px, const uint32_t* py,
                                                             const uint32_t* ur, const uint32_t* ug,
                                                             const uint32_t* gtab, uint32_t* ws, uint32_t* ox,
                                                             uint32_t* oy, uint32_t* flag) {
  __shared__ CoreLds L;
  const uint32_t i0 = blockIdx.x * WG + threadIdx.x;
  const uint32_t i = i0 < n ? i0 : n - 1;
  ge P;
  P.x = ld(px, i);
  P.y = ld(py, i);
  uint32_t a[8], b[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    a[k] = ur[(size_t)i * 8 + k];
    b[k] = ug[(size_t)i * 8 + k];
  }
  bool o1, o2;
  const sc sa = sc_from_limbs(a, o1), sb = sc_from_limbs(b, o2);
  gej Q;
  bool inf;
  ecmult_core(Q, inf, P, sa, sb, gtab, ws, L);
  const fe zi = fe_inv(Q.z);
  const fe zi2 = fe_sqr(zi);
  if (i0 < n) {
    st(ox, i, fe_mul(Q.x, zi2));
    st(oy, i, fe_mul(Q.y, fe_mul(zi2, zi)));
    flag[i] = inf ? 1u : 0u;
  }
}
}  // namespace eges

extern "C" int eges_selftest_ecmult(uint32_t n, const uint32_t* px, const uint32_t* py, const uint32_t* ur,
                                    const uint32_t* ug, uint32_t* ox, uint32_t* oy, uint32_t* flag) {
  using namespace eges;
  const size_t B = (size_t)n * 32;
  const uint32_t blocks = (n + WG - 1) / WG;
  uint32_t *dpx, *dpy, *dur, *dug, *dox, *doy, *dfl, *gtab, *ws;
  if (hipMalloc(&dpx, B) || hipMalloc(&dpy, B) || hipMalloc(&dur, B) || hipMalloc(&dug, B) || hipMalloc(&dox, B) ||
      hipMalloc(&doy, B) || hipMalloc(&dfl, (size_t)n * 4) || hipMalloc(&gtab, gtab_bytes()) ||
      hipMalloc(&ws, ws_bytes_per_block() * blocks))
    return -1;
  (void)hipMemcpy(dpx, px, B, hipMemcpyHostToDevice);
  (void)hipMemcpy(dpy, py, B, hipMemcpyHostToDevice);
  (void)hipMemcpy(dur, ur, B, hipMemcpyHostToDevice);
  (void)hipMemcpy(dug, ug, B, hipMemcpyHostToDevice);
  if (launch_init_gtab(gtab, 0) != hipSuccess) return -3;
  hipLaunchKernelGGL(selftest_ecmult_kernel, dim3(blocks), dim3(WG), 0, 0, n, dpx, dpy, dur, dug, gtab, ws, dox, doy,
                     dfl);
  hipError_t e = hipDeviceSynchronize();
  (void)hipMemcpy(ox, dox, B, hipMemcpyDeviceToHost);
  (void)hipMemcpy(oy, doy, B, hipMemcpyDeviceToHost);
  (void)hipMemcpy(flag, dfl, (size_t)n * 4, hipMemcpyDeviceToHost);
  (void)hipFree(dpx); (void)hipFree(dpy); (void)hipFree(dur); (void)hipFree(dug); (void)hipFree(dox);
  (void)hipFree(doy); (void)hipFree(dfl); (void)hipFree(gtab); (void)hipFree(ws);
  return e == hipSuccess ? 0 : -2;
}

// ---------------------------------------------------------------- op microbenchmarks
// Each lane runs `reps` iterations of one operation on register-resident data; the host
// launches 2 blocks of 256 per CU (the recover kernel's occupancy) and reports wall time.
namespace eges {
template <int OP>
__global__ void __launch_bounds__(256, 2) opbench_kernel(uint32_t* sink, int reps) {
  uint32_t seed = blockIdx.x * 256 + threadIdx.x + 1;
  uint32_t w[8];
  for (int k = 0; k < 8; ++k) w[k] = seed * 2654435761u + k * 40503u;
  fe a = fe_from_u256(w);
  for (int k = 0; k < 8; ++k) w[k] = w[k] * 747796405u + 1u;
  fe b = fe_from_u256(w);
  gej J;
  J.x = a; J.y = b; J.z = fe_normalize_weak(fe_add(a, b));
  ge q;
  q.x = b; q.y = a;
  sc s1, s2;
  for (int k = 0; k < 8; ++k) { s1.v[k] = w[k] >> 1; s2.v[k] = w[k] * 3u >> 1; }
  uint32_t acc = 0;
#pragma unroll 1
  for (int r = 0; r < reps; ++r) {
    if constexpr (OP == 0) a = fe_mul(a, b);
    else if constexpr (OP == 1) a = fe_sqr(a);
    else if constexpr (OP == 2) J = gej_double(J);
    else if constexpr (OP == 3) { bool hz, rz; J = gej_add_ge(J, q, hz, rz); acc += hz + rz; }
    else if constexpr (OP == 4) a = fe_normalize(fe_add(a, b));
    else if constexpr (OP == 5) a = fe_normalize_weak(fe_sub<2>(a, fe_add(b, b)));
    else if constexpr (OP == 6) s1 = sc_mul(s1, s2);
    else if constexpr (OP == 7) { bool z = fe_is_zero(a); acc += z; a = fe_normalize_weak(fe_add(a, b)); }
  }
  for (int k = 0; k < FE_LIMBS; ++k) acc += a.v[k] + J.x.v[k] + J.y.v[k] + J.z.v[k];
  for (int k = 0; k < 8; ++k) acc += s1.v[k];
  sink[blockIdx.x * 256 + threadIdx.x] = acc;
}
}  // namespace eges

// SIMD-cycles per lane-op at 2.4 GHz nominal: wall * 2.4e9 * (CUs * 4 SIMDs) / (lanes * reps)
extern "C" double eges_opbench(int op, int reps) {
  hipDeviceProp_t prop;
  (void)hipGetDeviceProperties(&prop, 0);
  const int blocks = prop.multiProcessorCount * 2;
  uint32_t* sink;
  if (hipMalloc(&sink, (size_t)blocks * 256 * 4) != hipSuccess) return -1;
  auto launch = [&](int r) {
    switch (op) {
      case 0: hipLaunchKernelGGL(eges::opbench_kernel<0>, dim3(blocks), dim3(256), 0, 0, sink, r); break;
      case 1: hipLaunchKernelGGL(eges::opbench_kernel<1>, dim3(blocks), dim3(256), 0, 0, sink, r); break;
      case 2: hipLaunchKernelGGL(eges::opbench_kernel<2>, dim3(blocks), dim3(256), 0, 0, sink, r); break;
      case 3: hipLaunchKernelGGL(eges::opbench_kernel<3>, dim3(blocks), dim3(256), 0, 0, sink, r); break;
      case 4: hipLaunchKernelGGL(eges::opbench_kernel<4>, dim3(blocks), dim3(256), 0, 0, sink, r); break;
      case 5: hipLaunchKernelGGL(eges::opbench_kernel<5>, dim3(blocks), dim3(256), 0, 0, sink, r); break;
      case 6: hipLaunchKernelGGL(eges::opbench_kernel<6>, dim3(blocks), dim3(256), 0, 0, sink, r); break;
      case 7: hipLaunchKernelGGL(eges::opbench_kernel<7>, dim3(blocks), dim3(256), 0, 0, sink, r); break;
    }
  };
  launch(8);
  (void)hipDeviceSynchronize();
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0, 0);
  launch(reps);
  (void)hipEventRecord(e1, 0);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  (void)hipFree(sink);
  const double lanes = (double)blocks * 256;
  return (double)ms * 2.4e6 * prop.multiProcessorCount * 4 / (lanes * reps);
}

// ---------------------------------------------------------------- row-form field (fr.cuh)
// One item per 16-lane row; canonical 256-bit words in and out, as eges_selftest.
#include "fr.cuh"
#include "frg.cuh"
#include "modinv_row.cuh"
namespace eges {
enum : int {
  FR_MUL = 0,      // a * b
  FR_SQR = 1,      // a^2
  FR_MULSUB = 2,   // a * b - 4c
  FR_SUB = 3,      // a - b
  FR_LAZY = 4,     // (2a) * (a + 2b) - 2b (a - b): magnitudes 2 x 3, fr_sub<1>
  FR_NORMW = 5,    // normalize_weak(7a) (limbs up to 7 * 2^29)
  FR_CHAIN = 6,    // 64 squarings of a, then * b
  FR_QUAD = 7,     // fr_mul4 (a*b, b*c, c*a, a*a in one pass): out = (ab + 2bc + 3ca) * a^2
  FR_QUAD2 = 8,    // fr_mul2 (a*b, c*c): out = ab + 2c^2
  FR_INV = 9,      // fr_inv_var (row-parallel safegcd): out = a^-1
  FR_GADD = 10,    // gejq_add of lift(a, even) on Z = c and lift(b, parity of c) on Z = c^2: x of the sum
  FR_SCINV = 11,   // sc_inv_row_var (row-parallel safegcd mod n) of a < n: out = a^-1 mod n
  FR_MULSUB_MAX = 12,  // (a + 2p') * (2b) - 8 (5c), 2p' = kconst<1> (limbs ~2^30, == 0 mod p): magnitudes
                       // 3 x 2 with the largest preset (M = 3, SH = 3), columns near their 2^64 bound
};
__global__ void fr_selftest_kernel(int op, uint32_t n, const uint32_t* A, const uint32_t* B, const uint32_t* C,
                                   uint32_t* out) {
  const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t item = gid >> 4;
  if (op >= FR_QUAD) item = gid >> 6;  // one item per wave: operands replicated in all rows
  const bool in = item < n;
  const uint32_t i = in ? item : 0;
  const fr a = fe_to_fr(ld(A, i)), b = fe_to_fr(ld(B, i)), c = fe_to_fr(ld(C, i));
  fr r;
  switch (op) {
    case FR_MUL: r = fr_mul(a, b); break;
    case FR_SQR: r = fr_sqr(a); break;
    case FR_MULSUB: r = fr_mul_sub<1, 2>(a, b, c); break;
    case FR_MULSUB_MAX: {
      const fr a3 = fr{a.v + kconst<1>()}, b2 = fr_add(b, b);
      const fr c5 = fr_add(c, fr_add(fr_add(c, c), fr_add(c, c)));
      r = fr_mul_sub<3, 3>(a3, b2, c5);
      break;
    }
    case FR_SUB: r = fr_sub<1>(a, b); break;
    case FR_LAZY: {
      const fr a2 = fr_add(a, a);
      const fr t = fr_add(a, fr_add(b, b));
      const fr u = fr_mul(a2, t);
      const fr w = fr_mul(fr_add(b, b), fr_sub<1>(a, b));
      r = fr_sub<1>(u, w);
      break;
    }
    case FR_NORMW: r = fr_normalize_weak(fr_mul_small(a, 7)); break;
    case FR_CHAIN: {
      fr t = a;
#pragma unroll 1
      for (int k = 0; k < 64; ++k) t = fr_sqr(t);
      r = fr_mul(t, b);
      break;
    }
    case FR_QUAD: {
      fr p0, p1, p2, p3;
      fr_mul4(p0, p1, p2, p3, a, b, b, c, c, a, a, a);
      r = fr_add(fr_add(p0, fr_mul_small(p1, 2)), fr_mul_small(p2, 3));
      r = fr_mul(r, p3);
      break;
    }
    case FR_QUAD2: {
      fr q0, q1;
      fr_mul2(q0, q1, a, b, c, c);
      r = fr_add(q0, fr_mul_small(q1, 2));
      break;
    }
    case FR_INV: r = fr_inv_var(a); break;
    case FR_GADD: {
      ger P, Q;
      ger_set_xo(P, fr_normalize(a), false);
      const bool odd = (__builtin_amdgcn_readlane(c.v, 0) & 1u) != 0;
      ger_set_xo(Q, fr_normalize(b), odd);
      const fr z1 = fr_normalize(c), z2 = fr_sqr(z1);
      gejr A, B;
      fr t1, t2, u1, u2;
      fr_mul2(t1, t2, z1, z1, z2, z2);  // Z1^2, Z2^2
      fr_mul4(A.x, A.y, B.x, B.y, P.x, t1, P.y, fr_mul(t1, z1), Q.x, t2, Q.y, fr_mul(t2, z2));
      (void)u1;
      (void)u2;
      A.z = z1;
      B.z = z2;
      bool rinf;
      const gejr S = gejq_add(A, false, B, false, rinf);
      const fr zi = fr_inv_var(S.z);
      r = rinf ? fr_zero() : fr_mul(S.x, fr_sqr(zi));
      break;
    }
    default: r = a;
  }
  uint32_t x[8];
  if (op == FR_SCINV) {  // a scalar in, a scalar out (the raw words, not reduced mod p)
    uint32_t w[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) w[k] = A[(size_t)i * 8 + k];
    bool ov;
    const sc si = sc_inv_row_var(sc_from_limbs(w, ov));
#pragma unroll
    for (int k = 0; k < 8; ++k) x[k] = si.v[k];
  } else {
    fe_to_u256(x, fe_normalize(fr_to_fe_row(r)));
  }
  if (in && (threadIdx.x & (op >= FR_QUAD ? 63 : 15)) == 0) {
#pragma unroll
    for (int k = 0; k < 8; ++k) out[(size_t)i * 8 + k] = x[k];
  }
}

// Inversion latency: one wave per CU, `reps` dependent row-form inversions (mode 0: fr_inv_var mod
// p, 1: sc_inv_row_var mod n) on a chain x -> (x + 1)^-1; mean s_memtime cycles per inversion.
__global__ void __launch_bounds__(64) inv_latency_kernel(int mode, int reps, uint64_t* cyc, uint32_t* sink) {
  uint32_t w[8];
  for (int k = 0; k < 8; ++k) w[k] = (blockIdx.x + 1) * 2654435761u + k * 40503u;
  w[7] &= 0x7FFFFFFFu;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  uint32_t acc = 0;
  if (mode == 0) {
    fr x = fe_to_fr(fe_from_u256(w));
#pragma unroll 1
    for (int r = 0; r < reps; ++r) x = fr_inv_var(fr_add(x, fr_one()));
    acc = x.v;
  } else {
    bool ov;
    sc x = sc_from_limbs(w, ov);
#pragma unroll 1
    for (int r = 0; r < reps; ++r) {
      x.v[0] += 1;  // (no carry: the chain only needs distinct nonzero values)
      x = sc_inv_row_var(x);
    }
    acc = x.v[0];
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  sink[blockIdx.x * 64 + threadIdx.x] = acc;
  if (threadIdx.x == 0) cyc[blockIdx.x] = (t1 - t0) / (uint64_t)reps;
}

// Latency microbenchmark: one wave per CU, each runs a chain of `reps` dependent squarings in
// lane-serial form (mode 0: fe_sqr, every lane its own chain) or row form (mode 1: fr_sqr).
__global__ void __launch_bounds__(64) fr_latency_kernel(int mode, int reps, uint32_t* sink) {
  uint32_t w[8];
  for (int k = 0; k < 8; ++k) w[k] = (blockIdx.x * 64 + threadIdx.x + 1) * 2654435761u + k * 40503u;
  fe a = fe_from_u256(w);
  uint32_t acc = 0;
  if (mode == 0) {
#pragma unroll 1
    for (int r = 0; r < reps; ++r) a = fe_sqr(a);
    for (int k = 0; k < FE_LIMBS; ++k) acc += a.v[k];
  } else {
    fr x = fe_to_fr(a);
#pragma unroll 1
    for (int r = 0; r < reps; ++r) x = fr_sqr(x);
    acc = x.v;
  }
  sink[blockIdx.x * 64 + threadIdx.x] = acc;
}
}  // namespace eges

extern "C" int eges_fr_selftest(int op, uint32_t n, const uint32_t* a, const uint32_t* b, const uint32_t* c,
                                uint32_t* out) {
  const size_t B = (size_t)n * 32;
  uint32_t *da, *db, *dc, *dout;
  if (hipMalloc(&da, B) || hipMalloc(&db, B) || hipMalloc(&dc, B) || hipMalloc(&dout, B)) return -1;
  (void)hipMemcpy(da, a, B, hipMemcpyHostToDevice);
  (void)hipMemcpy(db, b, B, hipMemcpyHostToDevice);
  (void)hipMemcpy(dc, c, B, hipMemcpyHostToDevice);
  const uint32_t lanes = (op >= eges::FR_QUAD ? 64u : 16u) * n;
  hipLaunchKernelGGL(eges::fr_selftest_kernel, dim3((lanes + 255) / 256), dim3(256), 0, 0, op, n, da, db, dc, dout);
  hipError_t e = hipDeviceSynchronize();
  (void)hipMemcpy(out, dout, B, hipMemcpyDeviceToHost);
  (void)hipFree(da); (void)hipFree(db); (void)hipFree(dc); (void)hipFree(dout);
  return e == hipSuccess ? 0 : -2;
}

// mean s_memtime cycles per dependent row-form inversion at one wave per CU (mode 0 mod p, 1 mod n)
extern "C" double eges_inv_latency(int mode, int reps) {
  hipDeviceProp_t prop;
  (void)hipGetDeviceProperties(&prop, 0);
  const int blocks = prop.multiProcessorCount;
  uint32_t* sink;
  uint64_t* cyc;
  if (hipMalloc(&sink, (size_t)blocks * 64 * 4) != hipSuccess || hipMalloc(&cyc, (size_t)blocks * 8) != hipSuccess)
    return -1;
  hipLaunchKernelGGL(eges::inv_latency_kernel, dim3(blocks), dim3(64), 0, 0, mode, reps, cyc, sink);
  if (hipDeviceSynchronize() != hipSuccess) return -2;
  std::vector<uint64_t> h(blocks);
  (void)hipMemcpy(h.data(), cyc, (size_t)blocks * 8, hipMemcpyDeviceToHost);
  (void)hipFree(sink);
  (void)hipFree(cyc);
  double s = 0;
  for (uint64_t v : h) s += (double)v;
  return s / blocks;
}

// ns per dependent squaring at one wave per CU (mode 0 lane-serial fe, 1 row-form fr)
extern "C" double eges_fr_latency(int mode, int reps) {
  hipDeviceProp_t prop;
  (void)hipGetDeviceProperties(&prop, 0);
  const int blocks = prop.multiProcessorCount;
  uint32_t* sink;
  if (hipMalloc(&sink, (size_t)blocks * 64 * 4) != hipSuccess) return -1;
  hipLaunchKernelGGL(eges::fr_latency_kernel, dim3(blocks), dim3(64), 0, 0, mode, 8, sink);
  (void)hipDeviceSynchronize();
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0, 0);
  hipLaunchKernelGGL(eges::fr_latency_kernel, dim3(blocks), dim3(64), 0, 0, mode, reps, sink);
  (void)hipEventRecord(e1, 0);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  (void)hipFree(sink);
  return (double)ms * 1e6 / reps;
}
