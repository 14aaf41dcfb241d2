// Static instruction counts of field-multiply variants:
// the engine's schoolbook product (fe.cuh fe_mul) against a one-level Karatsuba 5 + 4 split,
// both followed by the same reduction. Compile-only: tools/isa_count.sh prints the histograms.
#include "fe.cuh"
using namespace eges;

// a = a0 + a1 X, X = 2^(29*5): a0 b0 (25 MADs), a1 b1 (16), (a0 + a1)(b0 + b1) (25), then the
// middle columns minus both outer products (64-bit column subtractions)
DEV void cols_mul_kara(uint64_t S[17], const fe& a, const fe& b) {
  uint32_t as[5], bs[5];
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    as[i] = a.v[i] + (i < 4 ? a.v[5 + i] : 0u);
    bs[i] = b.v[i] + (i < 4 ? b.v[5 + i] : 0u);
  }
  uint64_t L[9], H[7], M[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) L[k] = 0, M[k] = 0;
#pragma unroll
  for (int k = 0; k < 7; ++k) H[k] = 0;
#pragma unroll
  for (int i = 0; i < 5; ++i)
#pragma unroll
    for (int j = 0; j < 5; ++j) {
      L[i + j] = mad64(a.v[i], b.v[j], L[i + j]);
      M[i + j] = mad64(as[i], bs[j], M[i + j]);
    }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) H[i + j] = mad64(a.v[5 + i], b.v[5 + j], H[i + j]);
#pragma unroll
  for (int k = 0; k < 17; ++k) S[k] = 0;
#pragma unroll
  for (int k = 0; k < 9; ++k) S[k] += L[k];
#pragma unroll
  for (int k = 0; k < 7; ++k) S[k + 10] += H[k];
#pragma unroll
  for (int k = 0; k < 9; ++k) S[k + 5] += M[k] - L[k] - (k < 7 ? H[k] : 0);
}

__global__ void k_mul_schoolbook(const fe* a, const fe* b, fe* o) {
  const int i = threadIdx.x;
  o[i] = fe_mul(a[i], b[i]);
}
__global__ void k_mul_karatsuba(const fe* a, const fe* b, fe* o) {
  const int i = threadIdx.x;
  uint64_t S[17];
  cols_mul_kara(S, a[i], b[i]);
  o[i] = fe_reduce_cols(S);
}
__global__ void k_sqr(const fe* a, fe* o) {
  const int i = threadIdx.x;
  o[i] = fe_sqr(a[i]);
}
