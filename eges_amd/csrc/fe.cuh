// Field arithmetic mod p = 2^256 - 2^32 - 977 for gfx950, radix 2^26 (10 limbs).
//
// Same values as libsecp256k1's field (crypto/secp256k1/libsecp256k1/src/field_10x26_impl.h,
// field_impl.h). The radix is chosen for the MI355X VALU, not copied: every 26x26-bit partial
// product (up to 28x28 with lazy additions) accumulates IN PLACE into a 64-bit column with one
// v_mad_u64_u32 (4.4 cyc / wave64 instruction, tools/ubench_valu.hip) — no carry flags, no
// zero-extension moves — and additions / subtractions are plain 32-bit v_add_u32 (2.5 cyc) on
// limbs with headroom. A full 32-bit-limb multiply instead needs a carry op per product.
//
// Representation: value = sum_k v[k] * 2^(26 k), k = 0..9 (up to 2^260). "Magnitude m": every
// limb <= m * 2^26 (+ a 2^19 slack on the outputs of mul/sqr/normalize_weak, which are
// magnitude 1). Inputs of fe_mul / fe_sqr must have magnitude <= 4; fe_sub<M>(a, b) needs
// magnitude(b) < 2M and returns magnitude(a) + 2M. Values are weak (congruent mod p, possibly
// >= p) until fe_normalize().
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define DEV __device__ __forceinline__

#include "modinv.cuh"

namespace eges {

struct fe {
  uint32_t v[10];
};

constexpr uint32_t M26 = 0x3FFFFFFu;
// 2^260 mod p = 2^36 + 15632  -> fold v * 2^260 as v * 15632 (same limb) + v * 2^10 (next limb)
constexpr uint32_t FOLD0 = 15632u;
constexpr uint32_t FOLD1 = 1024u;
// 2^256 mod p = 2^32 + 977 = 977 + 2^6 * 2^26
constexpr uint32_t C256_0 = 977u;
constexpr uint32_t C256_1 = 64u;

DEV uint64_t mad64(uint32_t a, uint32_t b, uint64_t c) { return (uint64_t)a * b + c; }

// A wave-uniform constant the optimiser cannot see through: keeps x * 2^k as ONE
// v_mad_u64_u32 (SGPR operand) instead of the v_mov + v_lshlrev_b64 + v_lshl_add_u64 the
// shift canonicalisation produces for 64-bit accumulators.
DEV uint32_t opaque_u32(uint32_t x) {
  asm volatile("" : "+s"(x));
  return x;
}

DEV fe fe_zero() {
  fe r;
#pragma unroll
  for (int i = 0; i < 10; ++i) r.v[i] = 0;
  return r;
}
DEV fe fe_one() { fe r = fe_zero(); r.v[0] = 1; return r; }
DEV fe fe_from_u32(uint32_t x) {  // x < 2^26 suffices for the constants used here
  fe r = fe_zero();
  r.v[0] = x & M26;
  r.v[1] = x >> 26;
  return r;
}

// 256-bit little-endian 32-bit limbs -> radix 2^26 (value unchanged, magnitude 1)
DEV fe fe_from_u256(const uint32_t x[8]) {
  fe r;
  r.v[0] = x[0] & M26;
  r.v[1] = ((x[0] >> 26) | (x[1] << 6)) & M26;
  r.v[2] = ((x[1] >> 20) | (x[2] << 12)) & M26;
  r.v[3] = ((x[2] >> 14) | (x[3] << 18)) & M26;
  r.v[4] = ((x[3] >> 8) | (x[4] << 24)) & M26;
  r.v[5] = (x[4] >> 2) & M26;
  r.v[6] = ((x[4] >> 28) | (x[5] << 4)) & M26;
  r.v[7] = ((x[5] >> 22) | (x[6] << 10)) & M26;
  r.v[8] = ((x[6] >> 16) | (x[7] << 16)) & M26;
  r.v[9] = x[7] >> 10;
  return r;
}

// Canonical (fully normalised) radix-2^26 -> 256-bit 32-bit limbs.
DEV void fe_to_u256(uint32_t x[8], const fe& a) {
  x[0] = a.v[0] | (a.v[1] << 26);
  x[1] = (a.v[1] >> 6) | (a.v[2] << 20);
  x[2] = (a.v[2] >> 12) | (a.v[3] << 14);
  x[3] = (a.v[3] >> 18) | (a.v[4] << 8);
  x[4] = (a.v[4] >> 24) | (a.v[5] << 2) | (a.v[6] << 28);
  x[5] = (a.v[6] >> 4) | (a.v[7] << 22);
  x[6] = (a.v[7] >> 10) | (a.v[8] << 16);
  x[7] = (a.v[8] >> 16) | (a.v[9] << 10);
}

// ------------------------------------------------------------------ reduction of 19 columns
// S[0..18]: column sums (each < 2^59.4). Returns magnitude-1 limbs.
DEV fe fe_reduce_cols(uint64_t S[19]) {
  const uint32_t f1 = opaque_u32(FOLD1), f16 = opaque_u32(1u << 16);
  // fold columns 18..10 (descending: column 18 spills into column 10, folded afterwards).
  // S_k 2^(26k) = (hi 2^32 + lo) 2^(26(k-10)) (2^36 + 15632)
#pragma unroll
  for (int k = 18; k >= 10; --k) {
    const uint32_t lo = (uint32_t)S[k];
    const uint32_t hi = (uint32_t)(S[k] >> 32);
    S[k - 10] = mad64(lo, FOLD0, S[k - 10]);
    S[k - 9] = mad64(lo, f1, S[k - 9]);
    S[k - 9] = mad64(hi, FOLD0 << 6, S[k - 9]);
    S[k - 8] = mad64(hi, f16, S[k - 8]);
  }
  fe r;
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    r.v[k] = (uint32_t)S[k] & M26;
    S[k + 1] += S[k] >> 26;
  }
  r.v[9] = (uint32_t)S[9] & M26;
  const uint64_t c = S[9] >> 26;  // < 2^33.5: multiple of 2^260
  const uint32_t cl = (uint32_t)c, ch = (uint32_t)(c >> 32);
  uint64_t t0 = mad64(cl, FOLD0, r.v[0]);
  uint64_t t1 = mad64(cl, f1, r.v[1]);
  t1 = mad64(ch, FOLD0 << 6, t1);
  r.v[0] = (uint32_t)t0 & M26;
  t1 += t0 >> 26;
  r.v[1] = (uint32_t)t1 & M26;
  r.v[2] += (uint32_t)(t1 >> 26) + (ch << 16);
  return r;
}

DEV fe fe_mul(const fe& a, const fe& b) {
  uint64_t S[19];
#pragma unroll
  for (int k = 0; k < 19; ++k) S[k] = 0;
#pragma unroll
  for (int i = 0; i < 10; ++i)
#pragma unroll
    for (int j = 0; j < 10; ++j) S[i + j] = mad64(a.v[i], b.v[j], S[i + j]);
  return fe_reduce_cols(S);
}

DEV fe fe_sqr(const fe& a) {
  uint32_t d[10];
#pragma unroll
  for (int i = 0; i < 10; ++i) d[i] = a.v[i] << 1;  // < 2^29.1 for magnitude <= 4
  uint64_t S[19];
#pragma unroll
  for (int k = 0; k < 19; ++k) S[k] = 0;
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    S[2 * i] = mad64(a.v[i], a.v[i], S[2 * i]);
#pragma unroll
    for (int j = i + 1; j < 10; ++j) S[i + j] = mad64(a.v[i], d[j], S[i + j]);
  }
  return fe_reduce_cols(S);
}

DEV fe fe_sqr_n(fe a, int n) {
#pragma unroll 1
  for (int i = 0; i < n; ++i) a = fe_sqr(a);
  return a;
}

// ------------------------------------------------------------------ linear ops (no carries)
DEV fe fe_add(const fe& a, const fe& b) {
  fe r;
#pragma unroll
  for (int i = 0; i < 10; ++i) r.v[i] = a.v[i] + b.v[i];
  return r;
}

// Limbs of K1 = a multiple of p whose every limb is ~2 * 2^26.
__constant__ const uint32_t FE_K1[10] = {0x7ff85e0u, 0x7fff7feu, 0x7fffffeu, 0x7fffffeu, 0x7fffffeu,
                                         0x7fffffeu, 0x7fffffeu, 0x7fffffeu, 0x7fffffeu, 0x7fffffeu};

// a - b for magnitude(b) < 2M; result magnitude(a) + 2M.
template <int M>
DEV fe fe_sub(const fe& a, const fe& b) {
  constexpr uint32_t k0 = 0x7ff85e0u * M, k1 = 0x7fff7feu * M, kk = 0x7fffffeu * M;
  fe r;
  r.v[0] = a.v[0] + k0 - b.v[0];
  r.v[1] = a.v[1] + k1 - b.v[1];
#pragma unroll
  for (int i = 2; i < 10; ++i) r.v[i] = a.v[i] + kk - b.v[i];
  return r;
}

template <int M>
DEV fe fe_neg(const fe& a) {
  return fe_sub<M>(fe_zero(), a);
}

// limbwise small multiple (magnitude * k)
DEV fe fe_mul_small(const fe& a, uint32_t k) {
  fe r;
#pragma unroll
  for (int i = 0; i < 10; ++i) r.v[i] = a.v[i] * k;
  return r;
}

// Carry pass: any magnitude (limbs < 2^32) -> magnitude 1 (same value mod p).
DEV fe fe_normalize_weak(const fe& a) {
  fe r;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const uint32_t t = a.v[i] + c;
    r.v[i] = t & M26;
    c = t >> 26;
  }
  const uint32_t t9 = a.v[9] + c;
  r.v[9] = t9 & M26;
  const uint32_t h = t9 >> 26;  // multiple of 2^260, < 2^7
  const uint32_t u0 = r.v[0] + h * FOLD0;
  r.v[0] = u0 & M26;
  r.v[1] += (u0 >> 26) + h * FOLD1;
  return r;
}

// Canonical representative in [0, p), any magnitude.
DEV fe fe_normalize(const fe& a) {
  fe r = fe_normalize_weak(a);  // < 2^260 + small
  // fold bits >= 2^256 (limb 9 bits 22..25): h * (2^32 + 977)
  uint32_t h = r.v[9] >> 22;
  r.v[9] &= 0x3FFFFFu;
  uint32_t c = h * C256_0;
  {
    uint32_t t = r.v[0] + c;
    r.v[0] = t & M26;
    t = r.v[1] + (t >> 26) + h * C256_1;
    r.v[1] = t & M26;
    c = t >> 26;
#pragma unroll
    for (int i = 2; i < 9; ++i) {
      t = r.v[i] + c;
      r.v[i] = t & M26;
      c = t >> 26;
    }
    r.v[9] += c;  // value now < 2^256 + 2^32 (r.v[9] <= 2^22)
  }
  // one more fold if it reached 2^256, then the value is < 2^33: no further carries past limb 2
  h = r.v[9] >> 22;
  r.v[9] &= 0x3FFFFFu;
  {
    uint32_t t = r.v[0] + h * C256_0;
    r.v[0] = t & M26;
    t = r.v[1] + (t >> 26) + h * C256_1;
    r.v[1] = t & M26;
    r.v[2] += t >> 26;
  }
  // r < 2^256; subtract p if r >= p  <=>  r + 2^32 + 977 >= 2^256
  uint32_t s[10];
  {
    uint32_t t = r.v[0] + C256_0;
    s[0] = t & M26;
    t = r.v[1] + (t >> 26) + C256_1;
    s[1] = t & M26;
    uint32_t cc = t >> 26;
#pragma unroll
    for (int i = 2; i < 10; ++i) {
      t = r.v[i] + cc;
      s[i] = t & M26;
      cc = t >> 26;
    }
    // s[9] bit 22 set <=> r + 2^32 + 977 >= 2^256
  }
  const bool ge = (s[9] >> 22) != 0;
  s[9] &= 0x3FFFFFu;
  fe o;
#pragma unroll
  for (int i = 0; i < 10; ++i) o.v[i] = ge ? s[i] : r.v[i];
  return o;
}

DEV bool fe_is_zero(const fe& a) {
  const fe n = fe_normalize(a);
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < 10; ++i) o |= n.v[i];
  return o == 0;
}

DEV bool fe_equal(const fe& a, const fe& b) { return fe_is_zero(fe_sub<1>(a, b)); }

DEV bool fe_is_odd(const fe& a) { return fe_normalize(a).v[0] & 1u; }

DEV fe fe_select(bool c, const fe& a, const fe& b) {
  fe r;
#pragma unroll
  for (int i = 0; i < 10; ++i) r.v[i] = c ? a.v[i] : b.v[i];
  return r;
}

// ---- exponentiation chains ------------------------------------------------
// a^(2^k - 1) ladder shared by sqrt and inverse: x2, x3, x6, x9, x11, x22, x44, x88, x176, x220, x223
struct fe_chain {
  fe x2, x3, x22, x223;
};

DEV fe_chain fe_chain_223(const fe& a) {
  fe_chain c;
  c.x2 = fe_mul(fe_sqr(a), a);
  c.x3 = fe_mul(fe_sqr(c.x2), a);
  fe x6 = fe_mul(fe_sqr_n(c.x3, 3), c.x3);
  fe x9 = fe_mul(fe_sqr_n(x6, 3), c.x3);
  fe x11 = fe_mul(fe_sqr_n(x9, 2), c.x2);
  c.x22 = fe_mul(fe_sqr_n(x11, 11), x11);
  fe x44 = fe_mul(fe_sqr_n(c.x22, 22), c.x22);
  fe x88 = fe_mul(fe_sqr_n(x44, 44), x44);
  fe x176 = fe_mul(fe_sqr_n(x88, 88), x88);
  fe x220 = fe_mul(fe_sqr_n(x176, 44), x44);
  c.x223 = fe_mul(fe_sqr_n(x220, 3), c.x3);
  return c;
}

// a^((p+1)/4); (p+1)/4 = 1^223 0 1^22 0000 11 00 (253 sqr, 13 mul).
// Returns whether the result squares back to a (field_impl.h:38-134 semantics).
DEV bool fe_sqrt(fe& r, const fe& a) {
  fe_chain c = fe_chain_223(a);
  fe t = fe_mul(fe_sqr_n(c.x223, 23), c.x22);
  t = fe_mul(fe_sqr_n(t, 6), c.x2);
  t = fe_sqr_n(t, 2);
  r = t;
  return fe_equal(fe_sqr(t), a);
}

// a^-1 (0 -> 0): constant-time safegcd (modinv.cuh) on the canonical value.
DEV fe fe_inv(const fe& a) {
  uint32_t x[8], y[8];
  fe_to_u256(x, fe_normalize(a));
  modinv256<ModP>(y, x);
  return fe_from_u256(y);
}

}  // namespace eges
