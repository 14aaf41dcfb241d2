#pragma once
// secp256k1 group law in row form (fr.cuh) for the latency kernel (k_recover_lat.hip).
//
// The same formulas, exceptional-case flags and magnitude bookkeeping as ge.cuh (dbl-2009-l
// doubling, madd-2007-bl mixed addition with the ADD_ZINV variant of group_impl.h:463-517,
// Meloni co-Z dblu / zaddu for the table, ge_set_xo_var group_impl.h:216-237), written over
// row-form field elements: every row of a wave holds one signature's point, every field
// product is limb-parallel over the row's lanes. Independent products of a formula are
// adjacent so the compiler can interleave their instruction streams (a latency-bound single
// wave per SIMD needs that ILP).
#include "fr.cuh"

namespace eges {

struct gejr {
  fr x, y, z;
};
struct ger {
  fr x, y;
};

DEV gejr gejr_double(const gejr& a) {
  const fr A = fr_sqr(a.x);
  const fr B = fr_sqr(a.y);
  const fr yz = fr_mul(a.y, a.z);
  const fr C = fr_sqr(B);
  const fr D = fr_sqr_sub<2>(fr_add(a.x, B), fr_add(A, C));  // (X+B)^2 - A - C = 2 X Y^2
  const fr E = fr_normalize_weak(fr_add(fr_add(A, A), A));   // 3 X^2
  gejr r;
  r.x = fr_sqr_sub<1, 2>(E, D);                               // E^2 - 4D
  const fr D2 = fr_add(D, D);
  r.y = fr_mul_sub<1, 3>(E, fr_sub<1>(D2, r.x), C);           // E (4XY^2 - X3) - 8C
  r.z = fr_add(yz, yz);
  return r;
}

// Mixed addition (ge.cuh gej_add_ge_t): PLAIN, or ZINV (b on the true curve, a on the table's
// isomorphic curve with global Z = *bzinv). CHECK computes h_zero (a == +-b) / r_zero.
template <AddMode M, bool CHECK = true>
DEV gejr gejr_add_ge_t(const gejr& a, const ger& b, const fr* bzinv, bool& h_zero, bool& r_zero) {
  const fr az = M == ADD_ZINV ? fr_mul(a.z, *bzinv) : a.z;
  const fr Z1Z1 = fr_sqr(az);
  const fr byz = fr_mul(b.y, az);
  const fr H = fr_mul_sub<1>(b.x, Z1Z1, a.x);
  const fr R = fr_mul_sub<2>(byz, Z1Z1, a.y);
  if (CHECK) {
    h_zero = fr_is_zero(H);
    r_zero = fr_is_zero(R);
  }
  const fr HH = fr_sqr(H);
  const fr zh = fr_mul(a.z, H);
  const fr HH2 = fr_add(HH, HH);
  const fr I = fr_add(HH2, HH2);
  const fr J = fr_mul(H, I);
  const fr V = fr_mul(a.x, I);
  const fr R2 = fr_add(R, R);
  gejr r;
  r.x = fr_sqr_sub<2>(R2, fr_add(J, fr_add(V, V)));
  const fr YJ = fr_mul(a.y, J);
  r.y = fr_mul_sub<1, 1>(R2, fr_sub<1>(V, r.x), YJ);
  r.z = fr_add(zh, zh);
  return r;
}

DEV void gejr_dblu(gejr& d, ger& p1, const ger& p) {
  const fr A = fr_sqr(p.x);
  const fr B = fr_sqr(p.y);
  const fr C = fr_sqr(B);
  const fr D = fr_sqr_sub<2>(fr_add(p.x, B), fr_add(A, C));
  const fr E = fr_normalize_weak(fr_add(fr_add(A, A), A));
  d.x = fr_sqr_sub<1, 2>(E, D);
  const fr D2 = fr_add(D, D);
  d.y = fr_mul_sub<1, 3>(E, fr_sub<1>(D2, d.x), C);
  d.z = fr_add(p.y, p.y);
  p1.x = fr_normalize_weak(D2);
  p1.y = fr_normalize_weak(fr_mul_small(fr_normalize_weak(fr_mul_small(C, 4)), 2));
}

DEV fr gejr_zaddu(ger& t, ger& b) {
  const fr dx = fr_normalize_weak(fr_sub<1>(t.x, b.x));
  const fr dy = fr_normalize_weak(fr_sub<1>(t.y, b.y));
  const fr A = fr_sqr(dx);
  const fr dy2 = fr_sqr(dy);
  const fr B = fr_mul(b.x, A);
  const fr C = fr_mul(t.x, A);
  const fr E = fr_mul(b.y, fr_sub<1>(C, B));
  t.x = fr_sub<2>(dy2, fr_add(B, C));
  t.x = fr_normalize_weak(t.x);
  t.y = fr_mul_sub<1>(dy, fr_sub<1>(B, t.x), E);
  b.x = B;
  b.y = E;
  return dx;
}

DEV gejr gejr_select(bool c, const gejr& a, const gejr& b) {
  gejr r;
  r.x = fr_select(c, a.x, b.x);
  r.y = fr_select(c, a.y, b.y);
  r.z = fr_select(c, a.z, b.z);
  return r;
}

// ---- square root and lift (field_impl.h:38-134, group_impl.h:216-237)
DEV fr fr_sqr_n(fr a, int n) {
#pragma unroll 1
  for (int i = 0; i < n; ++i) a = fr_sqr(a);
  return a;
}

// a^((p+1)/4) (253 sqr, 13 mul); true when it squares back to a
DEV bool fr_sqrt(fr& r, fr a) {
  const fr x2 = fr_mul(fr_sqr(a), a);
  const fr x3 = fr_mul(fr_sqr(x2), a);
  const fr x6 = fr_mul(fr_sqr_n(x3, 3), x3);
  const fr x9 = fr_mul(fr_sqr_n(x6, 3), x3);
  const fr x11 = fr_mul(fr_sqr_n(x9, 2), x2);
  const fr x22 = fr_mul(fr_sqr_n(x11, 11), x11);
  const fr x44 = fr_mul(fr_sqr_n(x22, 22), x22);
  const fr x88 = fr_mul(fr_sqr_n(x44, 44), x44);
  const fr x176 = fr_mul(fr_sqr_n(x88, 88), x88);
  const fr x220 = fr_mul(fr_sqr_n(x176, 44), x44);
  const fr x223 = fr_mul(fr_sqr_n(x220, 3), x3);
  fr t = fr_mul(fr_sqr_n(x223, 23), x22);
  t = fr_mul(fr_sqr_n(t, 6), x2);
  t = fr_sqr_n(t, 2);
  r = t;
  return fr_equal(fr_sqr(t), a);
}

// y from x (canonical or magnitude 1) with the requested parity; false for a non-residue.
// Returned coordinates are canonical.
DEV bool ger_set_xo(ger& r, fr x, bool odd) {
  const fr c = fr_add(fr_mul(fr_sqr(x), x), fr_small(7));
  fr y;
  const bool ok = fr_sqrt(y, c);
  fe yl = fe_normalize(fr_to_fe(y));
  const bool flip = ((yl.v[0] & 1u) != 0) != odd;
  yl = fe_select(flip, fe_normalize(fe_neg<1>(yl)), yl);
  r.x = fr_normalize(x);
  r.y = fe_to_fr(yl);
  return ok;
}

}  // namespace eges
