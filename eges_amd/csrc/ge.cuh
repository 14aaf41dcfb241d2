// secp256k1 group law on y^2 = x^3 + 7 for gfx950.
//
// Value-level restatement of libsecp256k1's group module (src/group_impl.h: gej_double_var
// :301-354, gej_add_ge_var :414-461, ge_set_xo_var :216-237, ge_is_valid_var :287-299).
// Formulas: doubling dbl-2009-l (2M + 5S), mixed addition madd-2007-bl (7M + 4S). The
// exceptional cases libsecp256k1 handles with branches (a == infinity, a == b, a == -b) are
// reported through flags so the kernel can resolve them with wave-uniform control flow.
#pragma once
#include "fe.cuh"

namespace eges {

struct gej {
  fe x, y, z;
};
struct ge {
  fe x, y;
};

// Jacobian doubling. Input with Z == 0 yields Z == 0 (infinity stays infinity).
DEV gej gej_double(const gej& a) {
  fe A = fe_sqr(a.x);
  fe B = fe_sqr(a.y);
  fe C = fe_sqr(B);
  fe t = fe_sqr(fe_add(a.x, B));
  t = fe_sub(fe_sub(t, A), C);
  fe D = fe_add(t, t);                     // 4 X Y^2
  fe E = fe_add(fe_add(A, A), A);          // 3 X^2
  fe F = fe_sqr(E);
  gej r;
  r.x = fe_sub(F, fe_add(D, D));           // E^2 - 2D
  fe C8 = fe_mul_small(C, 8);
  r.y = fe_sub(fe_mul(E, fe_sub(D, r.x)), C8);
  fe yz = fe_mul(a.y, a.z);
  r.z = fe_add(yz, yz);
  return r;
}

// Mixed addition a (Jacobian, not infinity) + b (affine). Sets h_zero when U2 == X1
// (a == +-b); then r_zero tells doubling (a == b) from infinity (a == -b) and the returned
// point is meaningless.
DEV gej gej_add_ge(const gej& a, const ge& b, bool& h_zero, bool& r_zero) {
  fe Z1Z1 = fe_sqr(a.z);
  fe U2 = fe_mul(b.x, Z1Z1);
  fe S2 = fe_mul(fe_mul(b.y, a.z), Z1Z1);
  fe H = fe_sub(U2, a.x);
  fe rr = fe_sub(S2, a.y);
  h_zero = fe_is_zero(H);
  r_zero = fe_is_zero(rr);
  fe HH = fe_sqr(H);
  fe I = fe_add(HH, HH);
  I = fe_add(I, I);                         // 4 HH
  fe J = fe_mul(H, I);
  rr = fe_add(rr, rr);                      // 2 (S2 - Y1)
  fe V = fe_mul(a.x, I);
  gej r;
  r.x = fe_sub(fe_sub(fe_sqr(rr), J), fe_add(V, V));
  fe YJ = fe_mul(a.y, J);
  r.y = fe_sub(fe_mul(rr, fe_sub(V, r.x)), fe_add(YJ, YJ));
  fe zh = fe_sqr(fe_add(a.z, H));
  r.z = fe_sub(fe_sub(zh, Z1Z1), HH);       // 2 Z1 H
  return r;
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

// y from x with the requested parity; false if x^3 + 7 is not a square (ge_set_xo_var).
DEV bool ge_set_xo(ge& r, const fe& x, bool odd) {
  fe c = fe_add(fe_mul(fe_sqr(x), x), fe_from_u32(7));
  fe y;
  bool ok = fe_sqrt(y, c);
  y = fe_normalize(y);
  bool flip = ((y.v[0] & 1u) != 0) != odd;
  y = fe_select(flip, fe_normalize(fe_neg(y)), y);
  r.x = x;
  r.y = y;
  return ok;
}

// On-curve check for an affine point with x, y < p (ge_is_valid_var).
DEV bool ge_is_valid(const ge& a) {
  fe y2 = fe_sqr(a.y);
  fe x3 = fe_add(fe_mul(fe_sqr(a.x), a.x), fe_from_u32(7));
  return fe_equal(y2, x3);
}

}  // namespace eges
