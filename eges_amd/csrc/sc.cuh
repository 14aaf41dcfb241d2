// Scalar arithmetic mod the group order n, and the GLV split used by the ecmult kernel.
//
// Values match libsecp256k1's scalar module (src/scalar_8x32_impl.h: set_b32 :165-179 reduces
// and reports overflow, is_high :220-236, negate :196; src/scalar_impl.h: inverse :55-255).
// Scalars are kept canonical (< n) at all times. The GLV decomposition is this engine's own
// (Babai rounding with constants derived from the curve); it only has to
// satisfy k1 + k2*lambda == k (mod n) with |k1|,|k2| < 2^129 — the recovered point, and hence
// every output byte, is independent of how k is split.
#pragma once
#include "fe.cuh"

namespace eges {

// 256x256 -> 512 schoolbook, row (operand) scanning over 32-bit limbs: each partial product
// is one v_mad_u64_u32 whose 64-bit addend carries the running limb.
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
#pragma unroll
  for (int i = 15; i > 0; --i) t[i] = (t[i] << 1) | (t[i - 1] >> 31);  // off-diagonal sum < 2^511
  t[0] <<= 1;
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

struct sc {
  uint32_t v[8];
};

// n, little-endian 32-bit limbs
__constant__ const uint32_t SC_N[8] = {0xD0364141u, 0xBFD25E8Cu, 0xAF48A03Bu, 0xBAAEDCE6u,
                                       0xFFFFFFFEu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
// 2^256 - n (129 bits)
constexpr uint32_t SC_NC0 = 0x2FC9BEBFu, SC_NC1 = 0x402DA173u, SC_NC2 = 0x50B75FC4u, SC_NC3 = 0x45512319u;
// floor(n/2)
__constant__ const uint32_t SC_HALF[8] = {0x681B20A0u, 0xDFE92F46u, 0x57A4501Du, 0x5D576E73u,
                                          0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0x7FFFFFFFu};

DEV sc sc_zero() { sc r; for (int i = 0; i < 8; ++i) r.v[i] = 0; return r; }
DEV sc sc_one() { sc r = sc_zero(); r.v[0] = 1; return r; }

DEV bool sc_is_zero(const sc& a) {
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) o |= a.v[i];
  return o == 0;
}

// a >= b (unsigned 256-bit compare)
DEV bool u256_ge(const uint32_t a[8], const uint32_t b[8]) {
  uint64_t br = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    uint64_t d = (uint64_t)a[i] - b[i] - br;
    br = (d >> 63) & 1;
  }
  return br == 0;
}

// r = a - b*(m), m in {0,1}, returns borrow
DEV uint32_t u256_sub_cond(uint32_t r[8], const uint32_t a[8], const uint32_t b[8], uint32_t m) {
  uint64_t br = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    uint64_t d = (uint64_t)a[i] - (b[i] & (0u - m)) - br;
    r[i] = (uint32_t)d;
    br = (d >> 63) & 1;
  }
  return (uint32_t)br;
}

// Reduce x (< 2^256 + small) given as 8 limbs + carry word into [0, n).
DEV sc sc_finalize(const uint32_t x[8], uint32_t carry) {
  sc r;
  // if carry: value = x + 2^256 ; subtract n once => x + (2^256 - n), fits in 256 bits when
  // x + 2^256 < 2n, which holds for our callers.
  uint32_t t[8];
  {
    uint64_t c = (uint64_t)x[0] + (SC_NC0 & (0u - carry));
    t[0] = (uint32_t)c; c >>= 32;
    c += (uint64_t)x[1] + (SC_NC1 & (0u - carry)); t[1] = (uint32_t)c; c >>= 32;
    c += (uint64_t)x[2] + (SC_NC2 & (0u - carry)); t[2] = (uint32_t)c; c >>= 32;
    c += (uint64_t)x[3] + (SC_NC3 & (0u - carry)); t[3] = (uint32_t)c; c >>= 32;
    c += (uint64_t)x[4] + carry; t[4] = (uint32_t)c; c >>= 32;
#pragma unroll
    for (int i = 5; i < 8; ++i) { c += x[i]; t[i] = (uint32_t)c; c >>= 32; }
  }
  uint32_t ge = u256_ge(t, SC_N) ? 1u : 0u;
  u256_sub_cond(r.v, t, SC_N, ge);
  return r;
}

// x[0..15] mod n. Three folds of hi * (2^256 - n).
DEV sc sc_reduce512(const uint32_t x[16]) {
  // stage 1: m = lo + hi * nc  (hi 8 limbs, nc 5 limbs incl. top 1) -> 13 limbs
  uint32_t m[13];
#pragma unroll
  for (int i = 0; i < 13; ++i) m[i] = i < 8 ? x[i] : 0;
  const uint32_t nc[5] = {SC_NC0, SC_NC1, SC_NC2, SC_NC3, 1u};
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    uint64_t c = 0;
#pragma unroll
    for (int j = 0; j < 5; ++j) {
      c = (uint64_t)x[8 + i] * nc[j] + (uint64_t)m[i + j] + (c >> 32);
      m[i + j] = (uint32_t)c;
    }
    // propagate
    uint64_t cc = c >> 32;
#pragma unroll
    for (int k = i + 5; k < 13; ++k) {
      cc += m[k];
      m[k] = (uint32_t)cc;
      cc >>= 32;
    }
  }
  // stage 2: m2 = m[0..7] + m[8..12] * nc -> 10 limbs
  uint32_t q[10];
#pragma unroll
  for (int i = 0; i < 10; ++i) q[i] = i < 8 ? m[i] : 0;
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    uint64_t c = 0;
#pragma unroll
    for (int j = 0; j < 5; ++j) {
      c = (uint64_t)m[8 + i] * nc[j] + (uint64_t)q[i + j] + (c >> 32);
      q[i + j] = (uint32_t)c;
    }
    uint64_t cc = c >> 32;
#pragma unroll
    for (int k = i + 5; k < 10; ++k) {
      cc += q[k];
      q[k] = (uint32_t)cc;
      cc >>= 32;
    }
  }
  // stage 3: q[8..9] is tiny (< 2^4); fold once more: r = q[0..7] + q[8..9]*nc
  uint32_t r8[8];
  uint64_t hi = (uint64_t)q[8] | ((uint64_t)q[9] << 32);
  {
    uint32_t h0 = (uint32_t)hi, h1 = (uint32_t)(hi >> 32);
    uint64_t c = (uint64_t)h0 * SC_NC0 + q[0];
    r8[0] = (uint32_t)c;
    c = (c >> 32) + (uint64_t)h0 * SC_NC1 + (uint64_t)h1 * SC_NC0 + q[1];
    r8[1] = (uint32_t)c;
    c = (c >> 32) + (uint64_t)h0 * SC_NC2 + (uint64_t)h1 * SC_NC1 + q[2];
    r8[2] = (uint32_t)c;
    c = (c >> 32) + (uint64_t)h0 * SC_NC3 + (uint64_t)h1 * SC_NC2 + q[3];
    r8[3] = (uint32_t)c;
    c = (c >> 32) + (uint64_t)h0 + (uint64_t)h1 * SC_NC3 + q[4];
    r8[4] = (uint32_t)c;
    c = (c >> 32) + (uint64_t)h1 + q[5];
    r8[5] = (uint32_t)c;
    c = (c >> 32) + q[6];
    r8[6] = (uint32_t)c;
    c = (c >> 32) + q[7];
    r8[7] = (uint32_t)c;
    c >>= 32;
    return sc_finalize(r8, (uint32_t)c);
  }
}

DEV sc sc_mul(const sc& a, const sc& b) {
  uint32_t t[16];
  mul_256x256(t, a.v, b.v);
  return sc_reduce512(t);
}

DEV sc sc_sqr(const sc& a) {
  uint32_t t[16];
  sqr_256(t, a.v);
  return sc_reduce512(t);
}

DEV sc sc_add(const sc& a, const sc& b) {
  uint32_t t[8];
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    c += (uint64_t)a.v[i] + b.v[i];
    t[i] = (uint32_t)c;
    c >>= 32;
  }
  return sc_finalize(t, (uint32_t)c);
}

DEV sc sc_neg(const sc& a) {
  sc r;
  uint32_t nz = sc_is_zero(a) ? 0u : 1u;
  uint64_t br = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    uint64_t d = (uint64_t)(SC_N[i] & (0u - nz)) - a.v[i] - br;
    r.v[i] = (uint32_t)d;
    br = (d >> 63) & 1;
  }
  return r;
}

DEV bool sc_is_high(const sc& a) {
  // a > n/2  <=>  !(n/2 >= a)
  return !u256_ge(SC_HALF, a.v);
}

DEV sc sc_select(bool c, const sc& a, const sc& b) {
  sc r;
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = c ? a.v[i] : b.v[i];
  return r;
}

// From 8 big-endian-derived limbs (already little-endian limb order): reduce mod n and
// report overflow (value >= n), as secp256k1_scalar_set_b32.
DEV sc sc_from_limbs(const uint32_t x[8], bool& overflow) {
  sc r;
  uint32_t ge = u256_ge(x, SC_N) ? 1u : 0u;
  overflow = ge != 0;
  u256_sub_cond(r.v, x, SC_N, ge);
  return r;
}

// a^-1 mod n (0 -> 0): constant-time safegcd (modinv.cuh).
DEV sc sc_inv(const sc& a) {
  sc r;
  modinv256<ModN>(r.v, a.v);
  return r;
}

// ---------------------------------------------------------------------------------
// GLV split: k = k1 + k2*lambda (mod n), |k1|,|k2| < 2^129, returned as sign + 160-bit
// magnitude. c1 = round(k*g1 / 2^384), c2 = round(k*g2 / 2^384);
// k1 = k - c1*a1 - c2*a2, k2 = c1*|b1| - c2*b2 (b1 < 0 < b2).
// Constants derived from lambda by the extended-Euclid lattice reduction.
// ---------------------------------------------------------------------------------
__constant__ const uint32_t GLV_G1[8] = {0x45DBB031u, 0xE893209Au, 0x71E8CA7Fu, 0x3DAA8A14u,
                                         0x9284EB15u, 0xE86C90E4u, 0xA7D46BCDu, 0x3086D221u};
__constant__ const uint32_t GLV_G2[8] = {0x8AC47F71u, 0x1571B4AEu, 0x9DF506C6u, 0x221208ACu,
                                         0x0ABFE4C4u, 0x6F547FA9u, 0x010E8828u, 0xE4437ED6u};
__constant__ const uint32_t GLV_A1[4] = {0x9284EB15u, 0xE86C90E4u, 0xA7D46BCDu, 0x3086D221u};
__constant__ const uint32_t GLV_B1[4] = {0x0ABFE4C3u, 0x6F547FA9u, 0x010E8828u, 0xE4437ED6u};  // |b1|
__constant__ const uint32_t GLV_A2[5] = {0x9D44CFD8u, 0x57C1108Du, 0xA8E2F3F6u, 0x14CA50F7u, 0x00000001u};
// b2 == a1

struct glv_half {
  uint32_t mag[5];  // |k| little-endian, < 2^129
  bool neg;
};

// c = round(k * g / 2^384), 128-bit result
DEV void glv_round(uint32_t c[4], const sc& k, const uint32_t g[8]) {
  uint32_t t[16];
  uint32_t gl[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) gl[i] = g[i];
  mul_256x256(t, k.v, gl);
  // add 2^383 then take bits 384..511
  uint64_t c0 = (uint64_t)t[11] + 0x80000000u;
  uint64_t carry = c0 >> 32;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    carry += t[12 + i];
    c[i] = (uint32_t)carry;
    carry >>= 32;
  }
}

// out (9 limbs, two's complement 288-bit) -= x (nx limbs) * y (ny limbs)
template <int NX, int NY>
DEV void sub_mul(uint32_t out[9], const uint32_t x[NX], const uint32_t y[NY]) {
  uint32_t p[NX + NY];
#pragma unroll
  for (int i = 0; i < NX + NY; ++i) p[i] = 0;
#pragma unroll
  for (int i = 0; i < NX; ++i) {
    uint64_t c = 0;
#pragma unroll
    for (int j = 0; j < NY; ++j) {
      c = (uint64_t)x[i] * y[j] + (uint64_t)p[i + j] + (c >> 32);
      p[i + j] = (uint32_t)c;
    }
    p[i + NY] = (uint32_t)(c >> 32);
  }
  uint64_t br = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    uint64_t d = (uint64_t)out[i] - (i < NX + NY ? p[i] : 0u) - br;
    out[i] = (uint32_t)d;
    br = (d >> 63) & 1;
  }
}

template <int NX, int NY>
DEV void add_mul(uint32_t out[9], const uint32_t x[NX], const uint32_t y[NY]) {
  uint32_t p[NX + NY];
#pragma unroll
  for (int i = 0; i < NX + NY; ++i) p[i] = 0;
#pragma unroll
  for (int i = 0; i < NX; ++i) {
    uint64_t c = 0;
#pragma unroll
    for (int j = 0; j < NY; ++j) {
      c = (uint64_t)x[i] * y[j] + (uint64_t)p[i + j] + (c >> 32);
      p[i + j] = (uint32_t)c;
    }
    p[i + NY] = (uint32_t)(c >> 32);
  }
  uint64_t cy = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    cy += (uint64_t)out[i] + (i < NX + NY ? p[i] : 0u);
    out[i] = (uint32_t)cy;
    cy >>= 32;
  }
}

DEV glv_half glv_to_half(const uint32_t v[9]) {
  glv_half h;
  h.neg = (v[8] >> 31) != 0;
  uint32_t m = h.neg ? 0xffffffffu : 0u;
  uint64_t c = h.neg ? 1u : 0u;
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    c += (uint64_t)(v[i] ^ m);
    h.mag[i] = (uint32_t)c;
    c >>= 32;
  }
  return h;
}

DEV void glv_split(glv_half& h1, glv_half& h2, const sc& k) {
  uint32_t c1[4], c2[4];
  uint32_t g1[8], g2[8], a1[4], b1[4], a2[5];
#pragma unroll
  for (int i = 0; i < 8; ++i) { g1[i] = GLV_G1[i]; g2[i] = GLV_G2[i]; }
#pragma unroll
  for (int i = 0; i < 4; ++i) { a1[i] = GLV_A1[i]; b1[i] = GLV_B1[i]; }
#pragma unroll
  for (int i = 0; i < 5; ++i) a2[i] = GLV_A2[i];
  glv_round(c1, k, g1);
  glv_round(c2, k, g2);
  uint32_t k1[9], k2[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) { k1[i] = i < 8 ? k.v[i] : 0; k2[i] = 0; }
  sub_mul<4, 4>(k1, c1, a1);
  sub_mul<4, 5>(k1, c2, a2);
  add_mul<4, 4>(k2, c1, b1);
  sub_mul<4, 4>(k2, c2, a1);  // b2 == a1
  h1 = glv_to_half(k1);
  h2 = glv_to_half(k2);
}

}  // namespace eges
