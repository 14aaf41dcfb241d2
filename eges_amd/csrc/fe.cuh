// Field arithmetic mod p = 2^256 - 2^32 - 977 for gfx950, radix 2^29 (9 limbs).
//
// Same values as libsecp256k1's field (crypto/secp256k1/libsecp256k1/src/field_10x26_impl.h,
// field_impl.h); the representation is this engine's own, chosen for the MI355X VALU: every
// 29x29-bit partial product accumulates IN PLACE into a 64-bit column with one
// v_mad_u64_u32 (a half-rate instruction, ~4.5 cycles per wave64 issue; tools/ubench_valu.hip)
// — no carry flags, no zero-extension moves — and additions / subtractions are full-rate 32-bit
// v_add_u32 / v_sub_u32 on limbs with 3 bits of headroom. 9 limbs need 81 partial products
// per multiply (radix 2^26: 100; 32-bit limbs: 64 products but a carry op for each).
//
// Representation: value = sum_k v[k] * 2^(29 k), k = 0..8 (up to 2^261). "Magnitude m": every
// limb <= m * (2^29 + 2^16). Outputs of fe_mul / fe_sqr / fe_normalize_weak have magnitude 1.
// Rules (each keeps every 64-bit column below 2^64 and every limb below 2^32):
//   fe_mul(a, b): m(a) * m(b) <= 6.5          fe_sqr(a): m(a) <= 2.5
//   fe_sub<M>(a, b): m(b) < 2M, result m(a) + 2M, which must stay <= 7 (so M <= 3)
//   any limb-wise sum: magnitude <= 7
// Values are weak (congruent mod p, possibly >= p) until fe_normalize().
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define DEV __device__ __forceinline__

#include "modinv.cuh"

namespace eges {

constexpr int FE_LIMBS = 9;

struct fe {
  uint32_t v[FE_LIMBS];
};

constexpr uint32_t M29 = 0x1FFFFFFFu;
// 2^261 mod p = 2^37 + 31264: fold v * 2^261 as v * 31264 (same limb) + v * 2^8 (next limb)
constexpr uint32_t FOLD0 = 31264u;
// 2^256 mod p = 2^32 + 977 = 977 + 2^3 * 2^29
constexpr uint32_t C256_0 = 977u;
constexpr uint32_t C256_1 = 8u;

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
  for (int i = 0; i < FE_LIMBS; ++i) r.v[i] = 0;
  return r;
}
DEV fe fe_one() { fe r = fe_zero(); r.v[0] = 1; return r; }
DEV fe fe_from_u32(uint32_t x) {
  fe r = fe_zero();
  r.v[0] = x & M29;
  r.v[1] = x >> 29;
  return r;
}

// 256-bit little-endian 32-bit limbs -> radix 2^29 (value unchanged, magnitude 1)
DEV fe fe_from_u256(const uint32_t x[8]) {
  fe r;
  r.v[0] = x[0] & M29;
  r.v[1] = ((x[0] >> 29) | (x[1] << 3)) & M29;
  r.v[2] = ((x[1] >> 26) | (x[2] << 6)) & M29;
  r.v[3] = ((x[2] >> 23) | (x[3] << 9)) & M29;
  r.v[4] = ((x[3] >> 20) | (x[4] << 12)) & M29;
  r.v[5] = ((x[4] >> 17) | (x[5] << 15)) & M29;
  r.v[6] = ((x[5] >> 14) | (x[6] << 18)) & M29;
  r.v[7] = ((x[6] >> 11) | (x[7] << 21)) & M29;
  r.v[8] = x[7] >> 8;
  return r;
}

// Canonical (fully normalised) radix-2^29 -> 256-bit 32-bit limbs.
DEV void fe_to_u256(uint32_t x[8], const fe& a) {
  x[0] = a.v[0] | (a.v[1] << 29);
  x[1] = (a.v[1] >> 3) | (a.v[2] << 26);
  x[2] = (a.v[2] >> 6) | (a.v[3] << 23);
  x[3] = (a.v[3] >> 9) | (a.v[4] << 20);
  x[4] = (a.v[4] >> 12) | (a.v[5] << 17);
  x[5] = (a.v[5] >> 15) | (a.v[6] << 14);
  x[6] = (a.v[6] >> 18) | (a.v[7] << 11);
  x[7] = (a.v[7] >> 21) | (a.v[8] << 8);
}

// ------------------------------------------------------------------ reduction of 17 columns
// S[0..16]: column sums (each < 2^63.9). Returns magnitude-1 limbs (limb 2 carries < 2^15 slack).
DEV fe fe_reduce_cols(uint64_t S[17]) {
  const uint32_t f8 = opaque_u32(1u << 8), f3 = opaque_u32(1u << 3);
  // Fold columns 9..16 into 0..8 with 2^261 == 2^37 + 31264 (mod p). S_k = hi 2^32 + lo:
  //   lo 2^(29k) = lo 2^(29(k-9)) (2^37 + 31264): two MADs into columns k-9, k-8;
  //   hi 2^32 2^(29k) either folds the same way (hi 8 31264 into k-8, hi 2^11 into k-7: two
  //   MADs) or moves up as 8 hi into column k+1 (one MAD) before that column is folded.
  // Every column pushes its hi up: 26 MADs, measured 6 % faster end to end than folding every hi
  // down (32 MADs) and 2.5 % faster than pushing from odd columns only (29 MADs) on the same box
  // — the serial chain costs nothing visible (both variants: profiles/r06/removed_ab_branches_r06.diff).
  // (The same push in the carry pass below, one MAD + 32-bit carry-in instead of a 64-bit
  // shift + add, measured 1 % slower; carries in two independent rounds instead of the serial
  // pass, for a single wave per SIMD, measured 12 % slower on the mid-size kernel's doubling
  // chain, r03: the chain is bound by issue, not by its dependences.)
  // Column 9 holds 8 products (< 2^63.7), so every pushed 8 hi < 2^35 keeps columns < 2^64.
#pragma unroll
  for (int k = 9; k <= 15; ++k) S[k + 1] = mad64((uint32_t)(S[k] >> 32), f3, S[k + 1]);  // push hi up
#pragma unroll
  for (int k = 9; k <= 15; ++k) {
    const uint32_t lo = (uint32_t)S[k];
    S[k - 9] = mad64(lo, FOLD0, S[k - 9]);
    S[k - 8] = mad64(lo, f8, S[k - 8]);
  }
  {
    // column 16: hi 2^32 2^(29*16) = 8 hi 2^(29*17), and
    // 2^(29*17) = 2^(29*8) 2^261 == 31264 2^(29*8) + 2^16 2^29 + 2^8 31264  (mod p)
    const uint32_t lo = (uint32_t)S[16];
    const uint32_t hi = (uint32_t)(S[16] >> 32);  // < 2^29
    S[7] = mad64(lo, FOLD0, S[7]);
    S[8] = mad64(lo, f8, S[8]);
    S[8] = mad64(hi, opaque_u32(FOLD0 << 3), S[8]);
    S[1] = mad64(hi, opaque_u32(1u << 19), S[1]);
    S[0] = mad64(hi, opaque_u32(FOLD0 << 11), S[0]);
  }
  fe r;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    r.v[k] = (uint32_t)S[k] & M29;
    S[k + 1] += S[k] >> 29;
  }
  r.v[8] = (uint32_t)S[8] & M29;
  const uint64_t c = S[8] >> 29;  // < 2^35: multiple of 2^261
  const uint32_t cl = (uint32_t)c, ch = (uint32_t)(c >> 32);
  const uint64_t t0 = mad64(cl, FOLD0, r.v[0]);
  uint64_t t1 = mad64(cl, f8, r.v[1]);
  t1 = mad64(ch, opaque_u32(FOLD0 << 3), t1);
  r.v[0] = (uint32_t)t0 & M29;
  t1 += t0 >> 29;
  r.v[1] = (uint32_t)t1 & M29;
  r.v[2] += (uint32_t)(t1 >> 29) + (ch << 11);
  return r;
}

// Column accumulation of a * b (81 MADs) / a^2 (45 MADs) on top of preset columns.
DEV void cols_mul(uint64_t S[17], const fe& a, const fe& b) {
#pragma unroll
  for (int i = 0; i < FE_LIMBS; ++i)
#pragma unroll
    for (int j = 0; j < FE_LIMBS; ++j) S[i + j] = mad64(a.v[i], b.v[j], S[i + j]);
}
DEV void cols_sqr(uint64_t S[17], const fe& a) {
  uint32_t d[FE_LIMBS];
#pragma unroll
  for (int i = 0; i < FE_LIMBS; ++i) d[i] = a.v[i] << 1;  // < 2^31.4 for magnitude <= 2.5
#pragma unroll
  for (int i = 0; i < FE_LIMBS; ++i) {
    S[2 * i] = mad64(a.v[i], a.v[i], S[2 * i]);
#pragma unroll
    for (int j = i + 1; j < FE_LIMBS; ++j) S[i + j] = mad64(a.v[i], d[j], S[i + j]);
  }
}
DEV void cols_zero(uint64_t S[17]) {
#pragma unroll
  for (int k = 0; k < 17; ++k) S[k] = 0;
}
// Columns preset to 2^SH * (M * 64p - c), c of magnitude < 2M: a product minus a linear term
// then costs 9 subtractions and shares the product's single carry pass (64p: see fe_sub).
template <int M, int SH>
DEV void cols_preset_sub(uint64_t S[17], const fe& c) {
  static_assert(M >= 1 && M <= 3 && SH >= 0 && SH <= 3, "cols_preset_sub");
  constexpr uint32_t k0 = 0x3FFF0BC0u * M, k1 = 0x3FFFFDFEu * M, kk = 0x3FFFFFFEu * M;
  S[0] = (uint64_t)(k0 - c.v[0]) << SH;
  S[1] = (uint64_t)(k1 - c.v[1]) << SH;
#pragma unroll
  for (int i = 2; i < FE_LIMBS; ++i) S[i] = (uint64_t)(kk - c.v[i]) << SH;
#pragma unroll
  for (int k = FE_LIMBS; k < 17; ++k) S[k] = 0;
}

DEV fe fe_mul(const fe& a, const fe& b) {
  uint64_t S[17];
  cols_zero(S);
  cols_mul(S, a, b);
  return fe_reduce_cols(S);
}

DEV fe fe_sqr(const fe& a) {
  uint64_t S[17];
  cols_zero(S);
  cols_sqr(S, a);
  return fe_reduce_cols(S);
}

// a * b - 2^SH * c and a^2 - 2^SH * c (magnitude(c) < 2M), magnitude-1 results.
template <int M, int SH = 0>
DEV fe fe_mul_sub(const fe& a, const fe& b, const fe& c) {
  uint64_t S[17];
  cols_preset_sub<M, SH>(S, c);
  cols_mul(S, a, b);
  return fe_reduce_cols(S);
}
template <int M, int SH = 0>
DEV fe fe_sqr_sub(const fe& a, const fe& c) {
  uint64_t S[17];
  cols_preset_sub<M, SH>(S, c);
  cols_sqr(S, a);
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
  for (int i = 0; i < FE_LIMBS; ++i) r.v[i] = a.v[i] + b.v[i];
  return r;
}

// a - b for magnitude(b) < 2M; result magnitude(a) + 2M. The subtrahend constant is 64p with
// every limb ~2^30 (= magnitude 2): limbs 2^30 - 62528, 2^30 - 514, 2^30 - 2 (x7).
template <int M>
DEV fe fe_sub(const fe& a, const fe& b) {
  static_assert(M >= 1 && M <= 3, "fe_sub: M in 1..3");
  constexpr uint32_t k0 = 0x3FFF0BC0u * M, k1 = 0x3FFFFDFEu * M, kk = 0x3FFFFFFEu * M;
  fe r;
  r.v[0] = a.v[0] + k0 - b.v[0];
  r.v[1] = a.v[1] + k1 - b.v[1];
#pragma unroll
  for (int i = 2; i < FE_LIMBS; ++i) r.v[i] = a.v[i] + kk - b.v[i];
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
  for (int i = 0; i < FE_LIMBS; ++i) r.v[i] = a.v[i] * k;
  return r;
}

// Carry pass: any limbs < 2^32 -> magnitude 1 (same value mod p).
DEV fe fe_normalize_weak(const fe& a) {
  fe r;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < FE_LIMBS - 1; ++i) {
    const uint32_t t = a.v[i] + c;
    r.v[i] = t & M29;
    c = t >> 29;
  }
  const uint32_t t8 = a.v[8] + c;
  r.v[8] = t8 & M29;
  const uint32_t h = t8 >> 29;  // multiple of 2^261, < 2^4
  const uint32_t u0 = r.v[0] + h * FOLD0;
  r.v[0] = u0 & M29;
  r.v[1] += (u0 >> 29) + (h << 8);
  return r;
}

// Canonical representative in [0, p), any magnitude.
DEV fe fe_normalize(const fe& a) {
  fe r = fe_normalize_weak(a);  // < 2^261 + small
  // fold bits >= 2^256 (limb 8 bits 24..28): h * (2^32 + 977)
  uint32_t h = r.v[8] >> 24;
  r.v[8] &= 0xFFFFFFu;
  {
    uint32_t t = r.v[0] + h * C256_0;
    r.v[0] = t & M29;
    t = r.v[1] + (t >> 29) + h * C256_1;
    r.v[1] = t & M29;
    uint32_t c = t >> 29;
#pragma unroll
    for (int i = 2; i < 8; ++i) {
      t = r.v[i] + c;
      r.v[i] = t & M29;
      c = t >> 29;
    }
    r.v[8] += c;  // value now < 2^256 + 2^35 (r.v[8] <= 2^24)
  }
  // one more fold if it reached 2^256; then the value is < 2^36: no carry past limb 1
  h = r.v[8] >> 24;
  r.v[8] &= 0xFFFFFFu;
  {
    uint32_t t = r.v[0] + h * C256_0;
    r.v[0] = t & M29;
    t = r.v[1] + (t >> 29) + h * C256_1;
    r.v[1] = t & M29;
    r.v[2] += t >> 29;
  }
  // r < 2^256; subtract p if r >= p  <=>  r + 2^32 + 977 >= 2^256
  uint32_t s[FE_LIMBS];
  {
    uint32_t t = r.v[0] + C256_0;
    s[0] = t & M29;
    t = r.v[1] + (t >> 29) + C256_1;
    s[1] = t & M29;
    uint32_t cc = t >> 29;
#pragma unroll
    for (int i = 2; i < FE_LIMBS; ++i) {
      t = r.v[i] + cc;
      s[i] = t & M29;
      cc = t >> 29;
    }
    // s[8] bit 24 set <=> r + 2^32 + 977 >= 2^256
  }
  const bool ge = (s[8] >> 24) != 0;
  s[8] &= 0xFFFFFFu;
  fe o;
#pragma unroll
  for (int i = 0; i < FE_LIMBS; ++i) o.v[i] = ge ? s[i] : r.v[i];
  return o;
}

DEV bool fe_is_zero(const fe& a) {
  const fe n = fe_normalize(a);
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < FE_LIMBS; ++i) o |= n.v[i];
  return o == 0;
}

DEV bool fe_equal(const fe& a, const fe& b) { return fe_is_zero(fe_sub<1>(a, b)); }

DEV bool fe_is_odd(const fe& a) { return fe_normalize(a).v[0] & 1u; }

DEV fe fe_select(bool c, const fe& a, const fe& b) {
  fe r;
#pragma unroll
  for (int i = 0; i < FE_LIMBS; ++i) r.v[i] = c ? a.v[i] : b.v[i];
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
