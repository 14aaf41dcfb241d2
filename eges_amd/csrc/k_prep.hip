// Table-initialisation and record-preparation kernels (gfx950).
#include "core.cuh"
#include "sender.cuh"

namespace eges {

// Fixed-base tables: gtab[t][e] = (e+1) * (t ? 2^128 G : G), affine, one record per entry.
// One thread per entry; simple double-and-add + inversion (runs once per device).
__global__ void __launch_bounds__(256) init_gtab_kernel(uint32_t* gtab) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 2 * GTAB) return;
  const int t = i / GTAB, e = i % GTAB;
  const uint32_t k = (uint32_t)e + 1;
  ge g;
  g.x = fe_const(t ? G128_X : GEN_X);
  g.y = fe_const(t ? G128_Y : GEN_Y);
  gej acc = gej_from_ge(g);
  int top = 31 - __clz(k);
  for (int b = top - 1; b >= 0; --b) {
    acc = gej_double(acc);
    if ((k >> b) & 1u) {
      bool hz, rz;
      acc = gej_add_ge(acc, g, hz, rz);  // m*B + B with 2 <= m < n-1: never exceptional
    }
  }
  fe zi = fe_inv(acc.z);
  fe zi2 = fe_sqr(zi);
  ge a;
  a.x = fe_normalize(fe_mul(acc.x, zi2));
  a.y = fe_normalize(fe_mul(acc.y, fe_mul(zi2, zi)));
  store_pt(gtab + (size_t)i * PT_WORDS, a);
}

// Comb table (core.cuh CBITS / CWIN / CTAB): gcomb[k][i] = (i + 1) 2^(16 k) G, affine; one
// thread per entry, double-and-add then 16 k doublings (never exceptional: multiples of G
// below n), once per device.
__global__ void __launch_bounds__(256) init_gcomb_kernel(uint32_t* gcomb) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= CWIN * CTAB) return;
  const int k = t / CTAB;
  const uint32_t m = (uint32_t)(t % CTAB) + 1;
  ge g;
  g.x = fe_const(GEN_X);
  g.y = fe_const(GEN_Y);
  gej acc = gej_from_ge(g);
  for (int b = 30 - __clz(m); b >= 0; --b) {
    acc = gej_double(acc);
    if ((m >> b) & 1u) {
      bool hz, rz;
      acc = gej_add_ge(acc, g, hz, rz);
    }
  }
  for (int d = 0; d < CBITS * k; ++d) acc = gej_double(acc);
  const fe zi = fe_inv(acc.z);
  const fe zi2 = fe_sqr(zi);
  ge a;
  a.x = fe_normalize(fe_mul(acc.x, zi2));
  a.y = fe_normalize(fe_mul(acc.y, fe_mul(zi2, zi)));
  store_pt(gcomb + (size_t)t * PT_WORDS, a);
}

// ------------------------------------------------------------------ prep kernels
// Record layout consumed by the recover kernel (SoA, stride n_pad words):
//   z[8], r[8], s[8] little-endian limbs of the raw 256-bit values; meta = recid | status << 8
__global__ void __launch_bounds__(256) prep_ecrecover_kernel(const uint8_t* __restrict__ msg,
                                                             const uint8_t* __restrict__ sig, uint32_t n,
                                                             uint32_t n_pad, uint32_t* __restrict__ rec) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t z[8], r[8], s[8];
  limbs_from_be32(z, msg + (size_t)i * 32);
  limbs_from_be32(r, sig + (size_t)i * 65);
  limbs_from_be32(s, sig + (size_t)i * 65 + 32);
  const uint32_t v = sig[(size_t)i * 65 + 64];
  // checkSignature (secp256.go:171-179): recid >= 4 => ErrInvalidRecoveryID
  const uint32_t meta = v >= 4 ? (ST_INVALID_RECOVERY_ID << 8) : v;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    rec[(size_t)k * n_pad + i] = z[k];
    rec[(size_t)(8 + k) * n_pad + i] = r[k];
    rec[(size_t)(16 + k) * n_pad + i] = s[k];
  }
  rec[(size_t)24 * n_pad + i] = meta;
}

// types.Sender classification (sender.cuh sender_meta) of the sender rows.
__global__ void __launch_bounds__(256) prep_sender_kernel(const uint8_t* __restrict__ sighash,
                                                          const uint8_t* __restrict__ rb,
                                                          const uint8_t* __restrict__ sb,
                                                          const uint8_t* __restrict__ vb,
                                                          const uint8_t* __restrict__ vflags, uint32_t n,
                                                          uint32_t n_pad, int signer, uint64_t chain_id,
                                                          uint32_t* __restrict__ rec) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t z[8], r[8], s[8], v[8];
  limbs_from_be32(z, sighash + (size_t)i * 32);
  limbs_from_be32(r, rb + (size_t)i * 32);
  limbs_from_be32(s, sb + (size_t)i * 32);
  limbs_from_be32(v, vb + (size_t)i * 32);
  const uint32_t meta = sender_meta(r, s, v, vflags ? vflags[i] : 0u, signer, chain_id);
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    rec[(size_t)k * n_pad + i] = z[k];
    rec[(size_t)(8 + k) * n_pad + i] = r[k];
    rec[(size_t)(16 + k) * n_pad + i] = s[k];
  }
  rec[(size_t)24 * n_pad + i] = meta;
}

// EVM ECRECOVER precompile (core/vm/contracts.go:77-101): input (hash, v, r, s), each 32 bytes,
// right-padded to 128 (common.RightPadBytes: bytes at or past inlen[i] read as zero). Rejected
// before the C call (-> nil output): input[32:63] not all zero, or ValidateSignatureValues(v =
// input[63] - 27 as a byte, r, s, homestead = false) fails (crypto.go:181-192).
__global__ void __launch_bounds__(256) prep_precompile_kernel(const uint8_t* __restrict__ input,
                                                              const uint32_t* __restrict__ inlen, uint32_t n,
                                                              uint32_t n_pad, uint32_t* __restrict__ rec) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint8_t* in = input + (size_t)i * 128;
  const uint32_t len = inlen ? inlen[i] : 128u;
  uint8_t b[128];
#pragma unroll
  for (int k = 0; k < 128; ++k) b[k] = (uint32_t)k < len ? in[k] : (uint8_t)0;
  uint32_t z[8], r[8], s[8];
  limbs_from_be32(z, b);
  limbs_from_be32(r, b + 64);
  limbs_from_be32(s, b + 96);
  uint32_t nz = 0;
#pragma unroll
  for (int k = 32; k < 63; ++k) nz |= b[k];
  const uint32_t v = (uint32_t)(uint8_t)(b[63] - 27u);
  bool r_zero = true, s_zero = true;
#pragma unroll
  for (int k = 0; k < 8; ++k) { r_zero = r_zero && r[k] == 0; s_zero = s_zero && s[k] == 0; }
  const bool bad = nz != 0 || r_zero || s_zero || u256_ge(r, SC_N) || u256_ge(s, SC_N) || v > 1u;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    rec[(size_t)k * n_pad + i] = z[k];
    rec[(size_t)(8 + k) * n_pad + i] = r[k];
    rec[(size_t)(16 + k) * n_pad + i] = s[k];
  }
  rec[(size_t)24 * n_pad + i] = bad ? (ST_INVALID_SIG << 8) : v;
}

// ------------------------------------------------------------------ launchers
hipError_t launch_init_gtab(uint32_t* gtab, hipStream_t st) {
  hipLaunchKernelGGL(init_gcomb_kernel, dim3((CWIN * CTAB + 255) / 256), dim3(256), 0, st,
                     gtab + (size_t)2 * GTAB * PT_WORDS);
  hipLaunchKernelGGL(init_gtab_kernel, dim3((2 * GTAB + 255) / 256), dim3(256), 0, st, gtab);
  return hipGetLastError();
}

hipError_t launch_prep_ecrecover(const uint8_t* msg, const uint8_t* sig, uint32_t n, uint32_t n_pad, uint32_t* rec,
                                 hipStream_t st) {
  hipLaunchKernelGGL(prep_ecrecover_kernel, dim3((n + 255) / 256), dim3(256), 0, st, msg, sig, n, n_pad, rec);
  return hipGetLastError();
}

hipError_t launch_prep_sender(const uint8_t* sighash, const uint8_t* r, const uint8_t* s, const uint8_t* v,
                              const uint8_t* vflags, uint32_t n, uint32_t n_pad, int signer, uint64_t chain_id,
                              uint32_t* rec, hipStream_t st) {
  hipLaunchKernelGGL(prep_sender_kernel, dim3((n + 255) / 256), dim3(256), 0, st, sighash, r, s, v, vflags, n, n_pad,
                     signer, chain_id, rec);
  return hipGetLastError();
}

hipError_t launch_prep_precompile(const uint8_t* input, const uint32_t* inlen, uint32_t n, uint32_t n_pad,
                                  uint32_t* rec, hipStream_t st) {
  hipLaunchKernelGGL(prep_precompile_kernel, dim3((n + 255) / 256), dim3(256), 0, st, input, inlen, n, n_pad, rec);
  return hipGetLastError();
}

size_t ws_bytes_per_block() { return WS_WORDS * sizeof(uint32_t); }
size_t gtab_bytes() { return ((size_t)2 * GTAB + (size_t)CWIN * CTAB) * PT_WORDS * sizeof(uint32_t); }
int threads_per_block() { return WG; }

}  // namespace eges
