#pragma once
// secp256k1 group law for the latency kernel (k_recover_lat.hip): one signature per wave,
// field elements in row form (fr.cuh) held replicated over the four rows, and every formula
// level's independent products computed together as one quad step (row r: product r).
//
// The formulas, exceptional-case flags and magnitude bookkeeping follow ge.cuh (dbl-2009-l
// doubling, madd-2007-bl mixed addition with the ADD_ZINV variant of group_impl.h:463-517,
// Meloni co-Z dblu / zaddu for the table, ge_set_xo_var group_impl.h:216-237). Levels:
//   doubling        2M + 5S in 3 quad steps  {X^2, Y^2, YZ} {B^2, (X+B)^2, E^2} {E (2D - X3)}
//   two doublings   in 5 quad steps (gejq_double2)
//   mixed addition  8M + 3S in 5 quad steps  {Z1^2, y2 Z1} {U2 - X1, S2 - Y1} {H^2, Z1 H, R^2}
//                                            {H I, X1 I} {R2 (V - X3), Y1 J}   (+1 for ZINV)
//   co-Z addition   4M + 2S in 4 quad steps
//   mixed addition after a doubling or a mixed addition: 3 quad steps (gejq_double_pre /
//   gejq_add_pre: its first two levels run in the previous operation's idle rows)
// where a lane-serial kernel pays one product after another.
#include "fr.cuh"

namespace eges {

struct gejr {
  fr x, y, z;
};
struct ger {
  fr x, y;
};

// In: X m1, Y <= 2, Z <= 2. Out: X, Y m1, Z m2. Z == 0 stays 0.
DEV gejr gejq_double(const gejr& a) {
  fr A, B, YZ;
  fr_mul3(A, B, YZ, a.x, a.x, a.y, a.y, a.y, a.z);
  const fr E = fr_normalize_weak(fr_add(fr_add(A, A), A));  // 3 X^2
  const fr XB = fr_add(a.x, B);
  fr C, T, F;
  fr_mul3(C, T, F, B, B, XB, XB, E, E);
  const fr D = fr_normalize_weak(fr_sub<2>(T, fr_add(A, C)));       // (X+B)^2 - A - C = 2 X Y^2
  gejr r;
  r.x = fr_normalize_weak(fr_sub<3>(F, fr_mul_small(D, 4)));        // E^2 - 4D
  r.y = fr_mul_sub<1, 3>(E, fr_sub<1>(fr_add(D, D), r.x), C);      // E (4XY^2 - X3) - 8C
  r.z = fr_add(YZ, YZ);                                             // 2 Y Z
  return r;
}

// Two doublings in 5 quad levels instead of 6. With U = 3X^3 formed beside Y^2, the doubling's
// Y3 = 3X^2 (4XY^2 - X3) - 8Y^4 is 3U (4Y^2 - U) - 8Y^4: one product one level after Y^2, so the
// second doubling's Y3 is ready in the same level as its X3 (gejq_double's E (2D - X3) waits a
// level for X3). Same values as gejq_double twice. In: X m1, Y <= 2, Z <= 2. Out: X, Y m1, Z m2.
//   {X^2, Y^2, YZ} {U, 2XY^2, E^2, Y^4} {Y', X'^2} {Y'^2, Y'Z', U', E'^2} {2X'Y'^2, 4Y'^4, 3U'(..)}
DEV gejr gejq_double2(const gejr& a) {
  fr A, B, YZ;
  fr_mul3(A, B, YZ, a.x, a.x, a.y, a.y, a.y, a.z);
  const fr E = fr_normalize_weak(fr_add(fr_add(A, A), A));  // 3 X^2
  fr U, T2, F, BB;
  fr_mul4(U, T2, F, BB, E, a.x, fr_add(a.x, a.x), B, E, E, B, B);  // 3X^3, 2XY^2, 9X^4, Y^4
  gejr h;
  h.x = fr_normalize_weak(fr_sub<3>(F, fr_mul_small(T2, 4)));       // 9X^4 - 8XY^2
  h.z = fr_add(YZ, YZ);                                             // 2 Y Z, m2
  const fr W = fr_normalize_weak(fr_sub<1>(fr_mul_small(B, 4), U));  // 4Y^2 - U
  // row 0: 3U W - 8 Y^4 (the subtraction preset into its columns); row 1: X'^2
  const uint64_t c0 = (uint64_t)rowsel(kconst<1>() - BB.v, 0u, 0u, 0u) << 3;
  fr A1;
  rep2(fr_mul_col(rowsel(fr_mul_small(U, 3), h.x, h.x, h.x), rowsel(W, h.x, h.x, h.x), c0), h.y, A1);
  // second doubling
  const fr E1 = fr_normalize_weak(fr_add(fr_add(A1, A1), A1));
  fr B1, YZ1, U1, F1;
  fr_mul4(B1, YZ1, U1, F1, h.y, h.y, h.y, h.z, E1, h.x, E1, E1);
  gejr r;
  r.z = fr_add(YZ1, YZ1);
  const fr W1 = fr_normalize_weak(fr_sub<1>(fr_mul_small(B1, 4), U1));
  fr T21, BB4, P;
  const fr B12 = fr_add(B1, B1);
  fr_mul3(T21, BB4, P, fr_add(h.x, h.x), B1, B12, B12, fr_mul_small(U1, 3), W1);  // 2X'Y'^2, 4Y'^4, 3U'W'
  r.x = fr_normalize_weak(fr_sub<3>(F1, fr_mul_small(T21, 4)));
  r.y = fr_normalize_weak(fr_sub<2>(P, fr_add(BB4, BB4)));         // 3U'W' - 8Y'^4
  return r;
}

// Mixed addition (ge.cuh gej_add_ge_t). a: X m1, Y <= 2, Z <= 2, not infinity; b: x m1, y <= 2.
// PLAIN: b in a's coordinates; ZINV: b on the true curve, a on the table's isomorphic curve
// with global Z = *bzinv. CHECK computes h_zero (a == +-b) and r_zero.
template <AddMode M, bool CHECK = true>
DEV gejr gejq_add_ge_t(const gejr& a, const ger& b, const fr* bzinv, bool& h_zero, bool& r_zero) {
  const fr az = M == ADD_ZINV ? fr_mul(a.z, *bzinv) : a.z;
  fr Z1Z1, byz;
  fr_mul2(Z1Z1, byz, az, az, b.y, az);
  // H = b.x Z1Z1 - X1 (row 0) and R = b.y Z1^3 - Y1 (row 1), subtrahends preset per row
  fr H, R;
  rep2(fr_mul_sub<2>(rowsel(b.x, byz, b.x, byz), Z1Z1, rowsel(a.x, a.y, a.x, a.y)), H, R);
  if (CHECK) {
    h_zero = fr_is_zero(H);
    r_zero = fr_is_zero(R);
  }
  fr HH, zh, RR;
  fr_mul3(HH, zh, RR, H, H, a.z, H, R, R);
  const fr HH2 = fr_add(HH, HH);
  const fr I = fr_add(HH2, HH2);                                      // 4 HH, m4
  fr J, V;
  fr_mul2(J, V, H, I, a.x, I);
  const fr R2sq = fr_normalize_weak(fr_mul_small(RR, 4));            // (2R)^2
  gejr r;
  r.x = fr_normalize_weak(fr_sub<2>(R2sq, fr_add(J, fr_add(V, V))));  // R2^2 - J - 2V
  const fr R2 = fr_add(R, R);
  fr W, YJ;
  fr_mul2(W, YJ, R2, fr_sub<1>(V, r.x), a.y, J);
  r.y = fr_normalize_weak(fr_sub<2>(W, fr_add(YJ, YJ)));             // R2 (V - X3) - 2 Y1 J
  r.z = fr_add(zh, zh);                                               // 2 Z1 H
  return r;
}

// ---- hoisted mixed additions (the latency kernels' Strauss windows). A doubling's last level
// has one product and a mixed addition's last two have two or three, so three rows idle. The
// first two levels of the next mixed addition (Z1^2, then H = x2 Z1^2 - X1 and Z1^3) depend only
// on the operation's Z3, X3 and the next point's x, so they run in those idle rows: a mixed
// addition after a doubling or after another mixed addition costs 3 quad levels instead of 5.
struct AddPre {
  fr h, z13;  // H = x2 Z1^2 - X1 (m1), Z1^3 (m1) of the addition that follows
};

// gejq_double, with the start of the mixed addition of a point with x = x2 to the result
DEV gejr gejq_double_pre(const gejr& a, const fr& x2, AddPre& pre) {
  fr A, B, YZ;
  fr_mul3(A, B, YZ, a.x, a.x, a.y, a.y, a.y, a.z);
  const fr E = fr_normalize_weak(fr_add(fr_add(A, A), A));  // 3 X^2
  const fr XB = fr_add(a.x, B);
  gejr r;
  r.z = fr_add(YZ, YZ);                                             // 2 Y Z, m2
  fr C, T, F, ZZ;
  fr_mul4(C, T, F, ZZ, B, B, XB, XB, E, E, r.z, r.z);
  const fr D = fr_normalize_weak(fr_sub<2>(T, fr_add(A, C)));       // 2 X Y^2
  r.x = fr_normalize_weak(fr_sub<3>(F, fr_mul_small(D, 4)));        // E^2 - 4D
  // row 0: E (2D - X3) - 8C (gejq_double's Y3); row 1: x2 Z3^2 - X3; row 2: Z3^3
  const uint32_t p32 = rowsel(kconst<1>() - C.v, kconst<1>() - r.x.v, 0u, 0u);
  const uint64_t col = (uint64_t)p32 << (row_id() == 0 ? 3 : 0);
  fr u;
  rep4(fr_mul_col(rowsel(E, x2, r.z, r.z), rowsel(fr_sub<1>(fr_add(D, D), r.x), ZZ, ZZ, ZZ), col), r.y, pre.h,
       pre.z13, u);
  return r;
}

// a + b (gejq_add_ge_t<ADD_PLAIN, false>'s values) from its hoisted start pre. NEXT: the idle rows
// also start the mixed addition of a point with x = x2n to the result (into nxt).
template <bool NEXT>
DEV gejr gejq_add_pre(const gejr& a, const ger& b, const AddPre& pre, const fr& x2n, AddPre& nxt) {
  // R = y2 Z1^3 - Y1 (row 0), H^2, Z1 H
  const uint64_t c1 = (uint64_t)rowsel(kconst<2>() - a.y.v, 0u, 0u, 0u);
  fr R, HH, zh, u;
  rep4(fr_mul_col(rowsel(b.y, pre.h, a.z, a.z), rowsel(pre.z13, pre.h, pre.h, pre.h), c1), R, HH, zh, u);
  const fr HH2 = fr_add(HH, HH);
  const fr I = fr_add(HH2, HH2);                                      // 4 HH, m4
  gejr r;
  r.z = fr_add(zh, zh);                                               // 2 Z1 H, m2
  fr RR, J, V, ZZ;
  if (NEXT) fr_mul4(RR, J, V, ZZ, R, R, pre.h, I, a.x, I, r.z, r.z);
  else fr_mul3(RR, J, V, R, R, pre.h, I, a.x, I);
  const fr R2sq = fr_normalize_weak(fr_mul_small(RR, 4));            // (2R)^2
  r.x = fr_normalize_weak(fr_sub<2>(R2sq, fr_add(J, fr_add(V, V))));  // R2^2 - J - 2V
  const fr R2 = fr_add(R, R);
  fr W, YJ;
  if (NEXT) {  // rows 2, 3: x2n Z3^2 - X3, Z3^3
    const uint64_t c3 = (uint64_t)rowsel(0u, 0u, kconst<1>() - r.x.v, 0u);
    rep4(fr_mul_col(rowsel(R2, a.y, x2n, r.z), rowsel(fr_sub<1>(V, r.x), J, ZZ, ZZ), c3), W, YJ, nxt.h, nxt.z13);
  } else {
    fr_mul2(W, YJ, R2, fr_sub<1>(V, r.x), a.y, J);
  }
  r.y = fr_normalize_weak(fr_sub<2>(W, fr_add(YJ, YJ)));             // R2 (V - X3) - 2 Y1 J
  return r;
}

// Start of the co-Z table: d = 2p in Jacobian with Z = 2y, and p1 = p on that same Z.
DEV void gejq_dblu(gejr& d, ger& p1, const ger& p) {
  fr A, B;
  fr_mul2(A, B, p.x, p.x, p.y, p.y);
  const fr E = fr_normalize_weak(fr_add(fr_add(A, A), A));
  const fr XB = fr_add(p.x, B);
  fr C, T, F;
  fr_mul3(C, T, F, B, B, XB, XB, E, E);
  const fr D = fr_normalize_weak(fr_sub<2>(T, fr_add(A, C)));  // 2 x y^2
  d.x = fr_normalize_weak(fr_sub<3>(F, fr_mul_small(D, 4)));
  d.y = fr_mul_sub<1, 3>(E, fr_sub<1>(fr_add(D, D), d.x), C);
  d.z = fr_add(p.y, p.y);
  p1.x = fr_normalize_weak(fr_add(D, D));                        // x (2y)^2 = 4 x y^2
  p1.y = fr_normalize_weak(fr_mul_small(fr_normalize_weak(fr_mul_small(C, 4)), 2));  // 8 y^4
}

// Co-Z addition with update (ge.cuh gej_zaddu): t <- t + b, b <- b, both on Z' = Z (X_t - X_b);
// returns Z'/Z. t == +-b is the caller's to exclude. X, Y magnitude 1 in and out.
DEV fr gejq_zaddu(ger& t, ger& b) {
  const fr dx = fr_normalize_weak(fr_sub<1>(t.x, b.x));
  const fr dy = fr_normalize_weak(fr_sub<1>(t.y, b.y));
  fr A, dy2;
  fr_mul2(A, dy2, dx, dx, dy, dy);
  fr B, C;
  fr_mul2(B, C, b.x, A, t.x, A);
  const fr E = fr_mul(b.y, fr_sub<1>(C, B));
  t.x = fr_normalize_weak(fr_sub<2>(dy2, fr_add(B, C)));
  t.y = fr_mul_sub<1>(dy, fr_sub<1>(B, t.x), E);
  b.x = B;
  b.y = E;
  return dx;
}

// General Jacobian addition a + b (add-2007-bl, 11M + 5S in 5 quad levels), both points in the
// same coordinates, with infinity flags in and out; wave-uniform exceptional cases resolved
// exactly (a == b doubles, a == -b is infinity). Used once per signature to join the partial
// sums of the wide latency kernel. In: X m1, Y <= 2, Z <= 2. Out: X, Y m1, Z m2. *exc (nullable)
// reports which exact branch ran: 0 none, 1 a == b, 2 a == -b.
DEV gejr gejq_add(const gejr& a, bool ainf, const gejr& b, bool binf, bool& rinf, int* exc = nullptr) {
  fr Z1Z1, Z2Z2, Y1Z2, Y2Z1;
  fr_mul4(Z1Z1, Z2Z2, Y1Z2, Y2Z1, a.z, a.z, b.z, b.z, a.y, b.z, b.y, a.z);
  fr U1, U2, S1, S2;
  fr_mul4(U1, U2, S1, S2, a.x, Z2Z2, b.x, Z1Z1, Y1Z2, Z2Z2, Y2Z1, Z1Z1);
  const fr H = fr_normalize_weak(fr_sub<1>(U2, U1));
  const fr Rd = fr_normalize_weak(fr_sub<1>(S2, S1));
  const fr H2 = fr_add(H, H), R2 = fr_add(Rd, Rd);  // r = 2 (S2 - S1)
  fr I, RR, Z1Z2;
  fr_mul3(I, RR, Z1Z2, H2, H2, R2, R2, a.z, b.z);   // (2H)^2, r^2, Z1 Z2
  fr J, V, ZH;
  fr_mul3(J, V, ZH, H, I, U1, I, Z1Z2, H);
  gejr r;
  r.x = fr_normalize_weak(fr_sub<2>(RR, fr_add(J, fr_add(V, V))));  // r^2 - J - 2V
  fr W, SJ;
  fr_mul2(W, SJ, R2, fr_sub<1>(V, r.x), S1, J);
  r.y = fr_normalize_weak(fr_sub<2>(W, fr_add(SJ, SJ)));             // r (V - X3) - 2 S1 J
  r.z = fr_add(ZH, ZH);                                               // 2 Z1 Z2 H
  rinf = false;
  if (exc) *exc = 0;
  if (ainf) {
    rinf = binf;
    return b;
  }
  if (binf) return a;
  if (fr_is_zero(H)) {  // same x: a == b or a == -b
    const bool dbl = fr_is_zero(Rd);
    if (exc) *exc = dbl ? 1 : 2;
    if (dbl) return gejq_double(a);
    rinf = true;
  }
  return r;
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

// y from x (magnitude 1) with the requested parity; false for a non-residue. Canonical out.
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
