// Constant-time modular inversion by Bernstein–Yang divsteps ("safegcd"), for gfx950.
//
// Replaces the Fermat exponentiations the reference uses for r^-1 mod n and Z^-1 mod p
// (libsecp256k1 src/scalar_impl.h:55-255, src/field_impl.h:136-224 in the vendored snapshot;
// same values). One inversion is 20 rounds of 30 divsteps on 32-bit words plus a 2x2
// transition-matrix update of the 270-bit signed state — about 15k VALU instructions, most of
// them full-rate 32-bit ops, against ~300k (scalar) / ~40k (field) for the exponentiations.
// Every lane runs the same instruction stream (no data-dependent branches), so it suits
// 64-lane wavefronts.
//
// Algorithm (D. J. Bernstein, B.-Y. Yang, "Fast constant-time gcd computation and modular
// inversion", TCHES 2019), in the zeta = -(delta + 1/2) form: state (zeta, f, g, d, e) with
// f = M, g = x, d = 0, e = 1. 590 divsteps suffice for 256-bit inputs; 20 x 30 = 600 are run.
// Afterwards g = 0, f = +-1 and x^-1 = +-d (mod M). Numbers are signed radix-2^30, 9 limbs.
//
// Attribution: divsteps_30 and update_de_30 below follow the structure of upstream
// libsecp256k1's src/modinv32_impl.h (secp256k1_modinv32_divsteps_30 / _update_de_30: the
// c1/c2 masks, the u/v/q/r transition matrix and the md/me correction by M^-1 mod 2^30),
// Copyright (c) 2020 Peter Dettman, Pieter Wuille, MIT License. That file is not part of the
// vendored reference snapshot (which predates it); the code here is written for gfx950.
#pragma once
#include <stdint.h>

#ifndef DEV
#define DEV __device__ __forceinline__
#endif

namespace eges {

struct s30 {
  int32_t v[9];
};

constexpr int32_t M30 = 0x3FFFFFFF;

// Modulus descriptors: limbs of M in radix 2^30 and M^-1 mod 2^30.
struct ModP {
  static constexpr int32_t m[9] = {0x3FFFFC2F, 0x3FFFFFFB, 0x3FFFFFFF, 0x3FFFFFFF, 0x3FFFFFFF,
                                   0x3FFFFFFF, 0x3FFFFFFF, 0x3FFFFFFF, 0xFFFF};
  static constexpr uint32_t minv = 0x2DDACACFu;
};
struct ModN {
  static constexpr int32_t m[9] = {0x10364141, 0x3F497A33, 0x348A03BB, 0x2BB739AB, 0x3FFFFEBA,
                                   0x3FFFFFFF, 0x3FFFFFFF, 0x3FFFFFFF, 0xFFFF};
  static constexpr uint32_t minv = 0x2A774EC1u;
};

struct trans2x2 {
  int32_t u, v, q, r;
};

// 30 divsteps on the low bits of f and g; returns the new zeta and the transition matrix
// scaled by 2^30.
DEV int32_t divsteps_30(int32_t zeta, uint32_t f0, uint32_t g0, trans2x2& t) {
  uint32_t u = 1, v = 0, q = 0, r = 1;
  uint32_t f = f0, g = g0;
#pragma unroll
  for (int i = 0; i < 30; ++i) {
    // c1 = -1 when zeta < 0, c2 = -1 when g is odd
    uint32_t c1 = (uint32_t)(zeta >> 31);
    const uint32_t c2 = 0u - (g & 1u);
    const uint32_t x = (f ^ c1) - c1, y = (u ^ c1) - c1, z = (v ^ c1) - c1;
    g += x & c2;
    q += y & c2;
    r += z & c2;
    c1 &= c2;  // swap when zeta < 0 and g odd
    zeta = (int32_t)(((uint32_t)zeta ^ c1) - 1u);
    f += g & c1;
    u += q & c1;
    v += r & c1;
    g >>= 1;
    u <<= 1;
    v <<= 1;
  }
  t.u = (int32_t)u;
  t.v = (int32_t)v;
  t.q = (int32_t)q;
  t.r = (int32_t)r;
  return zeta;
}

// [f, g] = t [f, g] / 2^30 (exact).
DEV void update_fg_30(s30& f, s30& g, const trans2x2& t) {
  int64_t cf = (int64_t)t.u * f.v[0] + (int64_t)t.v * g.v[0];
  int64_t cg = (int64_t)t.q * f.v[0] + (int64_t)t.r * g.v[0];
  cf >>= 30;
  cg >>= 30;
#pragma unroll
  for (int i = 1; i < 9; ++i) {
    const int32_t fi = f.v[i], gi = g.v[i];
    cf += (int64_t)t.u * fi + (int64_t)t.v * gi;
    cg += (int64_t)t.q * fi + (int64_t)t.r * gi;
    f.v[i - 1] = (int32_t)cf & M30;
    cf >>= 30;
    g.v[i - 1] = (int32_t)cg & M30;
    cg >>= 30;
  }
  f.v[8] = (int32_t)cf;
  g.v[8] = (int32_t)cg;
}

// [d, e] = (t [d, e] + M [md, me]) / 2^30 with md, me chosen so the division is exact.
// Keeps d, e in (-2M, M).
template <class Mod>
DEV void update_de_30(s30& d, s30& e, const trans2x2& t) {
  const int32_t sd = d.v[8] >> 31, se = e.v[8] >> 31;
  int32_t md = (t.u & sd) + (t.v & se);
  int32_t me = (t.q & sd) + (t.r & se);
  int64_t cd = (int64_t)t.u * d.v[0] + (int64_t)t.v * e.v[0];
  int64_t ce = (int64_t)t.q * d.v[0] + (int64_t)t.r * e.v[0];
  md -= (int32_t)((Mod::minv * (uint32_t)cd + (uint32_t)md) & (uint32_t)M30);
  me -= (int32_t)((Mod::minv * (uint32_t)ce + (uint32_t)me) & (uint32_t)M30);
  cd += (int64_t)Mod::m[0] * md;
  ce += (int64_t)Mod::m[0] * me;
  cd >>= 30;
  ce >>= 30;
#pragma unroll
  for (int i = 1; i < 9; ++i) {
    const int32_t di = d.v[i], ei = e.v[i];
    cd += (int64_t)t.u * di + (int64_t)t.v * ei;
    ce += (int64_t)t.q * di + (int64_t)t.r * ei;
    if (Mod::m[i] != 0) {
      cd += (int64_t)Mod::m[i] * md;
      ce += (int64_t)Mod::m[i] * me;
    }
    d.v[i - 1] = (int32_t)cd & M30;
    cd >>= 30;
    e.v[i - 1] = (int32_t)ce & M30;
    ce >>= 30;
  }
  d.v[8] = (int32_t)cd;
  e.v[8] = (int32_t)ce;
}

// r in (-2M, M) -> sign * r mod M in [0, M), sign < 0 meaning negate.
template <class Mod>
DEV void normalize_30(s30& r, int32_t sign) {
  int32_t add = r.v[8] >> 31;
#pragma unroll
  for (int i = 0; i < 9; ++i) r.v[i] += Mod::m[i] & add;
  const int32_t neg = sign >> 31;
#pragma unroll
  for (int i = 0; i < 9; ++i) r.v[i] = (r.v[i] ^ neg) - neg;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    r.v[i + 1] += r.v[i] >> 30;
    r.v[i] &= M30;
  }
  add = r.v[8] >> 31;
#pragma unroll
  for (int i = 0; i < 9; ++i) r.v[i] += Mod::m[i] & add;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    r.v[i + 1] += r.v[i] >> 30;
    r.v[i] &= M30;
  }
}

DEV s30 s30_from_u256(const uint32_t x[8]) {
  s30 r;
  r.v[0] = (int32_t)(x[0] & M30);
  r.v[1] = (int32_t)(((x[0] >> 30) | (x[1] << 2)) & M30);
  r.v[2] = (int32_t)(((x[1] >> 28) | (x[2] << 4)) & M30);
  r.v[3] = (int32_t)(((x[2] >> 26) | (x[3] << 6)) & M30);
  r.v[4] = (int32_t)(((x[3] >> 24) | (x[4] << 8)) & M30);
  r.v[5] = (int32_t)(((x[4] >> 22) | (x[5] << 10)) & M30);
  r.v[6] = (int32_t)(((x[5] >> 20) | (x[6] << 12)) & M30);
  r.v[7] = (int32_t)(((x[6] >> 18) | (x[7] << 14)) & M30);
  r.v[8] = (int32_t)(x[7] >> 16);
  return r;
}

// r in [0, 2^256) with limbs in [0, 2^30)
DEV void s30_to_u256(uint32_t x[8], const s30& a) {
  const uint32_t* v = reinterpret_cast<const uint32_t*>(a.v);
  x[0] = v[0] | (v[1] << 30);
  x[1] = (v[1] >> 2) | (v[2] << 28);
  x[2] = (v[2] >> 4) | (v[3] << 26);
  x[3] = (v[3] >> 6) | (v[4] << 24);
  x[4] = (v[4] >> 8) | (v[5] << 22);
  x[5] = (v[5] >> 10) | (v[6] << 20);
  x[6] = (v[6] >> 12) | (v[7] << 18);
  x[7] = (v[7] >> 14) | (v[8] << 16);
}

// x^-1 mod M for x in [0, M) as 8 little-endian 32-bit limbs (0 maps to 0).
template <class Mod>
DEV void modinv256(uint32_t out[8], const uint32_t x[8]) {
  s30 d, e, f, g;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    d.v[i] = 0;
    e.v[i] = i == 0 ? 1 : 0;
    f.v[i] = Mod::m[i];
  }
  g = s30_from_u256(x);
  int32_t zeta = -1;
#pragma unroll 1
  for (int it = 0; it < 20; ++it) {
    trans2x2 t;
    zeta = divsteps_30(zeta, (uint32_t)f.v[0], (uint32_t)g.v[0], t);
    update_de_30<Mod>(d, e, t);
    update_fg_30(f, g, t);
  }
  normalize_30<Mod>(d, f.v[8]);
  s30_to_u256(out, d);
}

}  // namespace eges
