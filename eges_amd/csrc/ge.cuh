// secp256k1 group law on y^2 = x^3 + 7 for gfx950.
//
// Value-level restatement of libsecp256k1's group module (src/group_impl.h: gej_double_var
// :301-354, gej_add_ge_var :414-461, ge_set_xo_var :216-237, ge_is_valid_var :287-299).
// Formulas: doubling dbl-2009-l (2M + 5S), mixed addition madd-2007-bl (8M + 3S here: Z3 = 2 Z1 H
// as a product keeps magnitudes in the radix-2^29 bounds);
// the table/accumulator "effective affine" trick follows ecmult_impl.h:52-110 (odd multiples
// on an isomorphic curve sharing one global Z). The
// exceptional cases libsecp256k1 handles with branches (a == infinity, a == b, a == -b) are
// reported through flags so the kernel can resolve them with wave-uniform control flow.
//
// Magnitudes (fe.cuh rules): at rest X, Y (and affine x) have magnitude 1, Z and affine y
// (after a conditional negation) at most 2; comments give the magnitude of each intermediate.
#pragma once
#include "fe.cuh"

namespace eges {

struct gej {
  fe x, y, z;
};
struct ge {
  fe x, y;
};

// Jacobian doubling (dbl-2009-l, 2M + 5S; the three "product - linear" steps fused into the
// product's reduction, fe_mul_sub). Input with Z == 0 yields Z == 0.
DEV gej gej_double(const gej& a) {
  const fe A = fe_sqr(a.x);                                   // 1
  const fe B = fe_sqr(a.y);                                   // 1
  const fe C = fe_sqr(B);                                     // 1
  const fe D = fe_sqr_sub<2>(fe_add(a.x, B), fe_add(A, C));   // (X+B)^2 - A - C = 2 X Y^2, 1
  const fe E = fe_normalize_weak(fe_add(fe_add(A, A), A));    // 3 X^2, 1
  gej r;
  r.x = fe_sqr_sub<1, 2>(E, D);                               // E^2 - 2 (2D), 1
  const fe D2 = fe_add(D, D);                                 // 4 X Y^2, 2
  r.y = fe_mul_sub<1, 3>(E, fe_sub<1>(D2, r.x), C);           // E (4XY^2 - X3) - 8C: 1 x 4, 1
  const fe yz = fe_mul(a.y, a.z);                             // <= 2 x <= 2 -> 1
  r.z = fe_add(yz, yz);                                       // 2 Y Z, 2
  return r;
}

// Mixed addition a (Jacobian, not infinity; Y may have magnitude 2) + b (affine, x magnitude 1,
// y magnitude <= 2).
// Sets h_zero when U2 == X1 (a == +-b); then r_zero tells doubling (a == b) from infinity
// (a == -b) and the returned point is meaningless.
//   ADD_PLAIN  b is affine in a's coordinates (madd-2007-bl; Z3 = 2 Z1 H as a product).
//   ADD_ZINV   b is affine on the true curve while a lives on the isomorphic curve of a table
//              with global Z = bzinv (a's true Jacobian Z is a.z * bzinv); the result stays in
//              a's coordinates (group_impl.h:463-517, gej_add_zinv_var; used at ecmult_impl.h:383). One extra mul.
//   ADD_ZR     as ADD_PLAIN, and *zr = Z3 / Z1 = 2H (group_impl.h:414-461, the rzr output).
//   CHECK      compute h_zero / r_zero. Without it an exceptional sum (H == 0) is not flagged
//              but still recognisable afterwards: Z3 = 2 Z1 H == 0, and every later doubling
//              or addition keeps Z == 0 (the accumulator is "poisoned"), so the caller can
//              detect it once at the end and redo the lane exactly (core.cuh ecmult_core).
enum AddMode { ADD_PLAIN, ADD_ZINV, ADD_ZR };
template <AddMode M, bool CHECK = true>
DEV gej gej_add_ge_t(const gej& a, const ge& b, const fe* bzinv, bool& h_zero, bool& r_zero, fe* zr) {
  const fe az = M == ADD_ZINV ? fe_mul(a.z, *bzinv) : a.z;           // <= 2
  const fe Z1Z1 = fe_sqr(az);                                        // 1
  const fe H = fe_mul_sub<1>(b.x, Z1Z1, a.x);                        // U2 - X1, 1
  const fe R = fe_mul_sub<2>(fe_mul(b.y, az), Z1Z1, a.y);            // S2 - Y1 (a.y <= 2), 1
  if (CHECK) {
    h_zero = fe_is_zero(H);
    r_zero = fe_is_zero(R);
  }
  const fe HH = fe_sqr(H);                                           // 1
  const fe HH2 = fe_add(HH, HH);
  const fe I = fe_add(HH2, HH2);                                     // 4 HH, 4
  const fe J = fe_mul(H, I);                                         // 1 x 4 -> 1
  const fe R2 = fe_add(R, R);                                        // 2 (S2 - Y1), 2
  const fe V = fe_mul(a.x, I);                                       // 1 x 4 -> 1
  gej r;
  r.x = fe_sqr_sub<2>(R2, fe_add(J, fe_add(V, V)));                  // R2^2 - J - 2V (3 < 4), 1
  const fe YJ = fe_mul(a.y, J);                                      // 1
  r.y = fe_mul_sub<1, 1>(R2, fe_sub<1>(V, r.x), YJ);                 // R2 (V - X3) - 2 Y1 J: 2 x 3, 1
  if (M == ADD_ZR) {
    *zr = fe_add(H, H);                                              // 2H, 2
    r.z = fe_mul(a.z, *zr);                                          // 2 x 2 -> 1
  } else {
    const fe zh = fe_mul(a.z, H);                                    // 2 x 1 -> 1
    r.z = fe_add(zh, zh);                                            // 2 Z1 H, 2
  }
  return r;
}
DEV gej gej_add_ge(const gej& a, const ge& b, bool& h_zero, bool& r_zero) {
  return gej_add_ge_t<ADD_PLAIN>(a, b, nullptr, h_zero, r_zero, nullptr);
}
DEV gej gej_add_ge_zinv(const gej& a, const ge& b, const fe& bzinv, bool& h_zero, bool& r_zero) {
  return gej_add_ge_t<ADD_ZINV>(a, b, &bzinv, h_zero, r_zero, nullptr);
}
DEV gej gej_add_ge_zr(const gej& a, const ge& b, fe& zr, bool& h_zero, bool& r_zero) {
  return gej_add_ge_t<ADD_ZR>(a, b, nullptr, h_zero, r_zero, &zr);
}
// Unchecked forms (see CHECK above).
DEV gej gej_add_ge_fast(const gej& a, const ge& b) {
  bool h, r;
  return gej_add_ge_t<ADD_PLAIN, false>(a, b, nullptr, h, r, nullptr);
}
DEV gej gej_add_ge_zinv_fast(const gej& a, const ge& b, const fe& bzinv) {
  bool h, r;
  return gej_add_ge_t<ADD_ZINV, false>(a, b, &bzinv, h, r, nullptr);
}
DEV gej gej_add_ge_zr_fast(const gej& a, const ge& b, fe& zr) {
  bool h, r;
  return gej_add_ge_t<ADD_ZR, false>(a, b, nullptr, h, r, &zr);
}

// ---- co-Z table building (Meloni, "New point addition formulae for ECC applications", 2007)
// Start from affine p: d = 2p in Jacobian with Z = 2y, and p1 = p on that same Z
// (p1 = (x (2y)^2, y (2y)^3) = (4xy^2, 8y^4), both by-products of the doubling). 1M + 5S.
// p.x magnitude 1, p.y magnitude 1.
DEV void gej_dblu(gej& d, ge& p1, const ge& p) {
  const fe A = fe_sqr(p.x);
  const fe B = fe_sqr(p.y);
  const fe C = fe_sqr(B);                                     // y^4
  const fe D = fe_sqr_sub<2>(fe_add(p.x, B), fe_add(A, C));   // 2 x y^2, 1
  const fe E = fe_normalize_weak(fe_add(fe_add(A, A), A));    // 3 x^2, 1
  d.x = fe_sqr_sub<1, 2>(E, D);                               // E^2 - 4D, 1
  const fe D2 = fe_add(D, D);                                 // 4 x y^2, 2
  d.y = fe_mul_sub<1, 3>(E, fe_sub<1>(D2, d.x), C);           // 1
  d.z = fe_add(p.y, p.y);                                     // 2y, 2
  p1.x = fe_normalize_weak(D2);                               // 1
  // 8 y^4 in two carry passes (8 x a magnitude-1 limb can exceed 32 bits)
  p1.y = fe_normalize_weak(fe_mul_small(fe_normalize_weak(fe_mul_small(C, 4)), 2));  // 1
}

// Co-Z addition with update (ZADDU): b and t share one Jacobian Z (only X, Y are held).
// t <- t + b and b <- b, both on Z' = Z (X_t - X_b); returns zr = Z' / Z. 4M + 2S.
// Exceptional (t == +-b) is the caller's to exclude. X, Y magnitude 1 in and out.
DEV fe gej_zaddu(ge& t, ge& b) {
  const fe dx = fe_normalize_weak(fe_sub<1>(t.x, b.x));      // 1
  const fe dy = fe_normalize_weak(fe_sub<1>(t.y, b.y));      // 1
  const fe A = fe_sqr(dx);
  const fe B = fe_mul(b.x, A);                                // X_b on Z'
  const fe C = fe_mul(t.x, A);
  const fe E = fe_mul(b.y, fe_sub<1>(C, B));                  // Y_b on Z': 1 x 3
  t.x = fe_sqr_sub<2>(dy, fe_add(B, C));                      // dy^2 - B - C, 1
  t.y = fe_mul_sub<1>(dy, fe_sub<1>(B, t.x), E);              // dy (B - X3) - E, 1
  b.x = B;
  b.y = E;
  return dx;
}

DEV gej gej_from_ge(const ge& b) {
  gej r;
  r.x = b.x;
  r.y = b.y;
  r.z = fe_one();
  return r;
}

DEV gej gej_select(bool c, const gej& a, const gej& b) {
  gej r;
  r.x = fe_select(c, a.x, b.x);
  r.y = fe_select(c, a.y, b.y);
  r.z = fe_select(c, a.z, b.z);
  return r;
}

// y from x (magnitude 1) with the requested parity; false if x^3 + 7 is not a square
// (ge_set_xo_var). Returned coordinates are canonical.
DEV bool ge_set_xo(ge& r, const fe& x, bool odd) {
  const fe c = fe_add(fe_mul(fe_sqr(x), x), fe_from_u32(7));        // 1 + tiny
  fe y;
  const bool ok = fe_sqrt(y, c);
  y = fe_normalize(y);
  const bool flip = ((y.v[0] & 1u) != 0) != odd;
  y = fe_select(flip, fe_normalize(fe_neg<1>(y)), y);
  r.x = fe_normalize(x);
  r.y = y;
  return ok;
}

// On-curve check for an affine point (ge_is_valid_var).
DEV bool ge_is_valid(const ge& a) {
  const fe y2 = fe_sqr(a.y);
  const fe x3 = fe_add(fe_mul(fe_sqr(a.x), a.x), fe_from_u32(7));
  return fe_equal(x3, y2);
}

}  // namespace eges
