// Field arithmetic mod p = 2^256 - 2^32 - 977 for gfx950.
//
// Same values as libsecp256k1's field (crypto/secp256k1/libsecp256k1/src/field_10x26_impl.h,
// field_impl.h), different representation: 8 x 32-bit little-endian limbs so that one
// v_mad_u64_u32 (measured 4.4 cyc/wave-inst, the same issue class as a 32-bit add with
// carry on gfx950; see tools/ubench_valu.hip) produces a full 32x32->64 partial product
// plus a 64-bit addend.
//
// Invariant ("weak" form): every fe holds a value < 2^256 that is congruent to the field
// element; it may be >= p. fe_normalize() maps it to [0, p). Equality / zero tests and
// serialisation normalise first.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define DEV __device__ __forceinline__

namespace eges {

struct fe {
  uint32_t v[8];
};

// 2^256 mod p = 2^32 + 977
constexpr uint32_t FE_C0 = 977u;

DEV fe fe_zero() { fe r; for (int i = 0; i < 8; ++i) r.v[i] = 0; return r; }
DEV fe fe_one() { fe r = fe_zero(); r.v[0] = 1; return r; }
DEV fe fe_from_u32(uint32_t x) { fe r = fe_zero(); r.v[0] = x; return r; }

// Fold a carry word k (value k * 2^256) back in: r += k * (2^32 + 977). k is small
// (< 2^34 here), so the fold can overflow 2^256 at most once more, by a tiny amount,
// which a second single-word fold absorbs without further carries.
DEV void fe_fold(fe& r, uint64_t k) {
  uint64_t c = (uint64_t)r.v[0] + (k & 0xffffffffull) * FE_C0;
  r.v[0] = (uint32_t)c;
  c = (c >> 32) + (uint64_t)r.v[1] + (k >> 32) * FE_C0 + (k & 0xffffffffull);
  r.v[1] = (uint32_t)c;
  c = (c >> 32) + (uint64_t)r.v[2] + (k >> 32);
  r.v[2] = (uint32_t)c;
  c >>= 32;
#pragma unroll
  for (int i = 3; i < 8; ++i) {
    c += r.v[i];
    r.v[i] = (uint32_t)c;
    c >>= 32;
  }
  // c is 0 or 1 here; if 1 the value wrapped to something < 2^35 and adding 2^32+977 cannot
  // carry beyond limb 1.
  uint64_t d = (uint64_t)r.v[0] + (uint32_t)c * FE_C0;
  r.v[0] = (uint32_t)d;
  d = (d >> 32) + (uint64_t)r.v[1] + (uint32_t)c;
  r.v[1] = (uint32_t)d;
  r.v[2] += (uint32_t)(d >> 32);
}

// r = lo + hi * 2^256 reduced to weak form. t[0..15] little-endian.
DEV fe fe_reduce512(const uint32_t t[16]) {
  fe r;
  // r = lo + hi * 977 + (hi << 32)
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    c += (uint64_t)t[8 + i] * FE_C0 + t[i];
    if (i > 0) c += t[8 + i - 1];
    r.v[i] = (uint32_t)c;
    c >>= 32;
  }
  c += t[15];  // top of (hi << 32)
  fe_fold(r, c);
  return r;
}

// 256x256 -> 512 schoolbook, row (operand) scanning: each partial product is one
// v_mad_u64_u32 whose 64-bit addend carries the running limb; the row carry is added
// as a 32-bit value.
DEV void mul_256x256(uint32_t t[16], const uint32_t a[8], const uint32_t b[8]) {
  uint64_t c = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    c = (uint64_t)a[0] * b[j] + (c >> 32);
    t[j] = (uint32_t)c;
  }
  t[8] = (uint32_t)(c >> 32);
#pragma unroll
  for (int i = 1; i < 8; ++i) {
    c = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      c = (uint64_t)a[i] * b[j] + (uint64_t)t[i + j] + (c >> 32);
      t[i + j] = (uint32_t)c;
    }
    t[i + 8] = (uint32_t)(c >> 32);
  }
}

// Squaring: off-diagonal products once, doubled, plus the diagonal.
DEV void sqr_256(uint32_t t[16], const uint32_t a[8]) {
#pragma unroll
  for (int i = 0; i < 16; ++i) t[i] = 0;
#pragma unroll
  for (int i = 0; i < 7; ++i) {
    uint64_t c = 0;
#pragma unroll
    for (int j = i + 1; j < 8; ++j) {
      c = (uint64_t)a[i] * a[j] + (uint64_t)t[i + j] + (c >> 32);
      t[i + j] = (uint32_t)c;
    }
    t[i + 8] = (uint32_t)(c >> 32);
  }
  // double
  uint32_t top = t[15] >> 31;
#pragma unroll
  for (int i = 15; i > 0; --i) t[i] = (t[i] << 1) | (t[i - 1] >> 31);
  t[0] <<= 1;
  (void)top;  // off-diagonal sum < 2^511, doubling cannot overflow 512 bits
  // add diagonal
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    uint64_t sq = (uint64_t)a[i] * a[i];
    c += (uint64_t)t[2 * i] + (uint32_t)sq;
    t[2 * i] = (uint32_t)c;
    c >>= 32;
    c += (uint64_t)t[2 * i + 1] + (uint32_t)(sq >> 32);
    t[2 * i + 1] = (uint32_t)c;
    c >>= 32;
  }
}

DEV fe fe_mul(const fe& a, const fe& b) {
  uint32_t t[16];
  mul_256x256(t, a.v, b.v);
  return fe_reduce512(t);
}

DEV fe fe_sqr(const fe& a) {
  uint32_t t[16];
  sqr_256(t, a.v);
  return fe_reduce512(t);
}

DEV fe fe_sqr_n(fe a, int n) {
#pragma unroll 1
  for (int i = 0; i < n; ++i) a = fe_sqr(a);
  return a;
}

DEV fe fe_add(const fe& a, const fe& b) {
  fe r;
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    c += (uint64_t)a.v[i] + b.v[i];
    r.v[i] = (uint32_t)c;
    c >>= 32;
  }
  // value = r + c*2^256 ; fold c (0/1)
  uint64_t d = (uint64_t)r.v[0] + (uint32_t)c * FE_C0;
  r.v[0] = (uint32_t)d;
  d = (d >> 32) + (uint64_t)r.v[1] + (uint32_t)c;
  r.v[1] = (uint32_t)d;
  d >>= 32;
#pragma unroll
  for (int i = 2; i < 8; ++i) {
    d += r.v[i];
    r.v[i] = (uint32_t)d;
    d >>= 32;
  }
  // second wrap only if r was >= 2^256 - 2^32 - 977; then the result is < 2^33 and
  // the fold below cannot carry past limb 1.
  uint64_t e = (uint64_t)r.v[0] + (uint32_t)d * FE_C0;
  r.v[0] = (uint32_t)e;
  e = (e >> 32) + (uint64_t)r.v[1] + (uint32_t)d;
  r.v[1] = (uint32_t)e;
  r.v[2] += (uint32_t)(e >> 32);
  return r;
}

// a - b (mod p): on borrow, subtract 2^32+977 (== add p, mod 2^256); a second borrow
// means the intermediate wrapped below zero again, subtract once more.
DEV fe fe_sub(const fe& a, const fe& b) {
  fe r;
  uint64_t br = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    uint64_t d = (uint64_t)a.v[i] - b.v[i] - br;
    r.v[i] = (uint32_t)d;
    br = (d >> 63) & 1;
  }
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    uint32_t m = (uint32_t)br;  // 1 if we must subtract 2^32 + 977
    uint64_t d = (uint64_t)r.v[0] - (uint64_t)(m * FE_C0);
    r.v[0] = (uint32_t)d;
    uint64_t b2 = (d >> 63) & 1;
    d = (uint64_t)r.v[1] - m - b2;
    r.v[1] = (uint32_t)d;
    b2 = (d >> 63) & 1;
#pragma unroll
    for (int i = 2; i < 8; ++i) {
      d = (uint64_t)r.v[i] - b2;
      r.v[i] = (uint32_t)d;
      b2 = (d >> 63) & 1;
    }
    br = b2 & m;
  }
  return r;
}

DEV fe fe_neg(const fe& a) { return fe_sub(fe_zero(), a); }

// r = a * k for a small constant k (< 2^30)
DEV fe fe_mul_small(const fe& a, uint32_t k) {
  fe r;
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    c = (uint64_t)a.v[i] * k + (c >> 32);
    r.v[i] = (uint32_t)c;
  }
  fe_fold(r, c >> 32);
  return r;
}

// Canonical representative in [0, p).
DEV fe fe_normalize(const fe& a) {
  // a >= p  <=>  a + (2^32 + 977) >= 2^256
  fe t;
  uint64_t c = (uint64_t)a.v[0] + FE_C0;
  t.v[0] = (uint32_t)c;
  c = (c >> 32) + (uint64_t)a.v[1] + 1u;
  t.v[1] = (uint32_t)c;
  c >>= 32;
#pragma unroll
  for (int i = 2; i < 8; ++i) {
    c += a.v[i];
    t.v[i] = (uint32_t)c;
    c >>= 32;
  }
  fe r;
  bool ge = c != 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = ge ? t.v[i] : a.v[i];
  return r;
}

DEV bool fe_is_zero(const fe& a) {
  fe n = fe_normalize(a);
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) o |= n.v[i];
  return o == 0;
}

DEV bool fe_equal(const fe& a, const fe& b) { return fe_is_zero(fe_sub(a, b)); }

DEV bool fe_is_odd(const fe& a) { return fe_normalize(a).v[0] & 1; }

DEV fe fe_select(bool c, const fe& a, const fe& b) {
  fe r;
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = c ? a.v[i] : b.v[i];
  return r;
}

// Big-endian 32-byte load; returns false if the value is >= p (field_10x26_impl.h:323-345).
DEV bool fe_set_b32_checked(fe& r, const uint8_t* b) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint8_t* q = b + 28 - 4 * i;
    r.v[i] = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | q[3];
  }
  fe n = fe_normalize(r);
  bool ok = true;
#pragma unroll
  for (int i = 0; i < 8; ++i) ok = ok && (n.v[i] == r.v[i]);
  return ok;
}

// ---- exponentiation chains ------------------------------------------------
// a^(2^k - 1) ladder shared by sqrt and inverse:
// x2, x3, x6, x9, x11, x22, x44, x88, x176, x220, x223
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

// a^(p-2); p-2 = 1^223 0 1^22 0000 1 0 11 0 1 (255 sqr, 15 mul).
DEV fe fe_inv(const fe& a) {
  fe_chain c = fe_chain_223(a);
  fe t = fe_mul(fe_sqr_n(c.x223, 23), c.x22);
  t = fe_mul(fe_sqr_n(t, 5), a);
  t = fe_mul(fe_sqr_n(t, 3), c.x2);
  t = fe_mul(fe_sqr_n(t, 2), a);
  return t;
}

}  // namespace eges
