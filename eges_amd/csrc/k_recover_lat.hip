// Latency kernels for small batches: one signature per wave (recover; verify at the end).
//
// Same path and same outputs as recover_kernel (k_recover.hip; recovery/main_impl.h:38-191,
// ecmult_impl.h:286-404, eckey_impl.h:36-52, crypto.go:194-197), for batches too small to fill
// the GPU with one signature per lane: there, a signature costs one lane's serial chain
// (~0.78 ms for a 1000-transaction block on 16 of 1024 SIMDs). Here a signature has a whole
// wave: every field product is limb-parallel over a 16-lane row (fr.cuh), and the four rows
// compute the independent products of each formula level together (quad steps, frg.cuh), so
// a 1000-signature block spreads over 1000 waves and each signature's chain is ~4x shorter.
//
//   parse, x = r (+n), c = x^3 + 7 ........ R' = (c x, c^2): R's image on E': y^2 = x^3 + 7 c^3
//                                            (no square root on wave 0's path)
//   r^-1, u1 = -z/r, u2 = s/r, GLV split .. wave 1 (scalar ALU + limb-parallel safegcd)
//   table {1..16}R' on one global Z ...... co-Z dblu / zaddu + backward rescale (as core.cuh)
//   Strauss over 26 windows (u2 R') ...... unchecked adds, exact redo if the accumulator was
//                                            poisoned (Z == 0 and not infinity)
//   u1 G by a comb table ................. wave 1, beside the Strauss loop
//   y = sqrt(c) .......................... narrow form: lane-serial root-helper workgroups at the
//                                            head of the launch (root_helper / root_fetch);
//                                            split form: wave 1
//   back to E: (X, Y, Z) -> (X, Y, Z y); + u1 G; Z^-1 (limb-parallel safegcd), affine,
//   serialize, Keccak address across the wave's lanes (keccak_wave.cuh); lane 0 stores.
// Forms: narrow (two waves per signature), split (four waves: the doubling chain cut at window
// SPLIT_W0, its high part on waves 2 / 3 against tables of D = 2^75 R'; batches up to
// EGES_LAT_WIDE_MAX = 256) and three-wave (the chain cut at TRI_W0, the high part of both GLV
// halves on wave 2, the roots from the helper workgroups; batches up to EGES_LAT_TRI_MAX).
// DESIGN.md §3.3.
#include <atomic>
#include <cstdlib>
#include <type_traits>

#include "core.cuh"
#include "frg.cuh"
#include "handoff.cuh"
#include "keccak_wave.cuh"
#include "modinv_row.cuh"
#include "sender.cuh"

namespace eges {

// One signature per workgroup of two waves (narrow form); the split form has four (LAT_WG_SPLIT).
constexpr int LAT_WG = 128;
// k doublings of a (the unchecked chains: Strauss windows, D = 2^k R')
DEV gejr gejq_double_n(gejr a, int k) {
#pragma unroll 1
  for (; k >= 2; k -= 2) a = gejq_double2(a);
#pragma unroll 1
  for (; k > 0; --k) a = gejq_double(a);
  return a;
}
constexpr int LAT_STAGE = 512;  // wire form: encodings up to this size decode out of LDS
// Split form: windows [0, SPLIT_W0) of both GLV halves against the R' table on wave 0, windows
// [SPLIT_W0, RWIN) against a table of D = 2^(RBITS SPLIT_W0) R' on waves 2 (R) and 3 (lambda R).
constexpr int SPLIT_W0 = 15;
static_assert(SPLIT_W0 > 0 && SPLIT_W0 < RWIN, "split point");
// the high part (bits from RBITS * SPLIT_W0 up, < 2^(130 - RBITS SPLIT_W0) with the recoding
// carry) in signed 4-bit windows against an 8-entry table of D: half the table build of a
// 16-entry one for a few more additions on the high waves' chain
constexpr int HBITS = 4;
constexpr int HTAB = 1 << (HBITS - 1);
constexpr int HWIN = (130 - RBITS * SPLIT_W0 + HBITS) / HBITS;
// Three-wave form: windows [0, TRI_W0) of both halves on wave 0, the rest of both halves on
// wave 2 against one table of D = 2^(RBITS TRI_W0) R' (and its beta x), so the two chains
// (table + TRI_W0 windows / RBITS TRI_W0 doublings + D's table + TRI_HWIN windows) are about even.
constexpr int TRI_W0 = 20;
static_assert(TRI_W0 > 0 && TRI_W0 < RWIN, "three-wave split point");
constexpr int TRI_HWIN = (130 - RBITS * TRI_W0 + HBITS) / HBITS;
static_assert(TRI_HWIN <= HWIN, "the high digits fit LatLds::hdig");
// forms of the latency kernels (RecoverParams::wide)
enum { FORM_NARROW = 0, FORM_SPLIT = 1, FORM_TRI = 2 };

// LDS flags of the split and three-wave forms (set once by their producer wave, polled by the
// consumers; the three-wave form uses F_DIG, F_G and F_HI)
enum { F_DIG = 0, F_Y, F_G, F_LHI, F_HI, F_ERR, NFLAGS };

struct LatLds {
  uint32_t tab[PTAB][2][16];  // {1..16} * R' (x, y), row form (all four rows read the same words)
  uint32_t zr[PTAB][16];      // Z ratios while the table is built (then their cubes)
  uint32_t zq[PTAB][16];      //   and their squares
  uint32_t btab[PTAB][16];    // beta x of the table entries (the lambda R' additions)
  uint32_t dtab[2][HTAB][2][16];  // split form: {1..8} * D, one copy per high-part wave
  uint32_t dzr[2][HTAB][16];
  uint32_t dzq[2][HTAB][16];
  uint32_t dbtab[HTAB][16];       //   and beta x for the lambda half (wave 3)
  int8_t rdig[2][RWIN];       // R / lambda R window digits
  int8_t hdig[2][HWIN];       // split form: the high parts in 4-bit windows
  uint16_t cdig[CWIN];        // comb digits of u_g
  uint32_t part[5][3][16];    // partial sums (X, Y, Z): [2] u_g G, [3] high parts, [4] lambda high part
  uint32_t pinf[5];           //   and their infinity flags
  uint32_t ylift[16];         // y of R (the square root, from the helper wave)
  uint32_t yok;
  uint32_t flag[NFLAGS];
  uint32_t skip;              // tests only: 1 + the flag this workgroup's producer skips (ho_skip)
  uint64_t w1t[2];            // diagnostic build: wave 1's r^-1 and u1 / u2 / GLV / digits ticks
  uint8_t stage[LAT_STAGE];   // wire form: the transaction's encoding
};

// Producer / consumer hand-off between the waves of one workgroup through LDS (split form,
// handoff.cuh): the producer's LDS writes are ordered before the flag by the release fence;
// consumers poll, bounded; a failed hand-off makes wave 0 write ST_ENGINE_FAULT.
DEV void flag_set(LatLds& S, int k) { ho_set(&S.flag[k], 1u, S.skip == (uint32_t)k + 1u); }
DEV void flag_wait(LatLds& S, int k) { (void)ho_wait<1>(&S.flag[k], 1u, &S.flag[F_ERR]); }

// signed fixed-window recoding (core.cuh recode) into this row's digit array
template <int W, int NW, class D>
DEV void recode_row(const glv_half& h, D* out) {
  uint32_t m[5];
#pragma unroll
  for (int i = 0; i < 5; ++i) m[i] = h.mag[i];
  int carry = 0;
#pragma unroll 1
  for (int w = 0; w < NW; ++w) {
    int v = (int)(m[0] & ((1u << W) - 1)) + carry;
    carry = v > (1 << (W - 1)) ? 1 : 0;
    v -= carry << W;
    out[w] = (D)(h.neg ? -v : v);  // every lane writes the same value
#pragma unroll
    for (int i = 0; i < 4; ++i) m[i] = (m[i] >> W) | (m[i + 1] << (32 - W));
    m[4] >>= W;
  }
}

DEV ger lds_pt(const uint32_t (*e)[16]) {
  const uint32_t L = row_lane();
  ger p;
  p.x.v = e[0][L];
  p.y.v = e[1][L];
  return p;
}
DEV void lds_put_pt(uint32_t (*e)[16], const ger& p) {
  const uint32_t L = row_lane();
  e[0][L] = p.x.v;
  e[1][L] = p.y.v;
}
// fixed-base table record (core.cuh layout: 9 limbs of x, 9 of y, 2 pad) -> row form
DEV ger gtab_pt(const uint32_t* rec) {
  const uint32_t L = row_lane();
  const uint32_t k = L <= 8 ? L : 8u;
  const uint32_t x = rec[k], y = rec[FE_LIMBS + k];
  ger p;
  p.x.v = L <= 8 ? x : 0u;
  p.y.v = L <= 8 ? y : 0u;
  return p;
}

DEV ger ger_neg_if(const ger& p, bool neg) {
  ger r;
  r.x = p.x;
  r.y = fr_select(neg, fr_neg<1>(p.y), p.y);
  return r;
}

// acc += p (core.cuh add_step / add_step_fast, quad form; inf is wave-uniform)
template <bool CHECKED>
DEV void add_r(gejr& acc, bool& inf, const ger& p, bool use, const Diag& dg) {
  gejr s;
  bool to_inf = false;
  if (CHECKED) {
    bool hz, rz;
    s = gejq_add_ge_t<ADD_PLAIN, true>(acc, p, nullptr, hz, rz);
    const bool exc = use && !inf && hz;
    if (__any(exc)) {
      diag_bump(dg, EGES_DIAG_LAT_EXC);
      s = gejr_select(exc && rz, gejq_double(acc), s);
    }
    to_inf = exc && !rz;
  } else {
    bool h, r;
    s = gejq_add_ge_t<ADD_PLAIN, false>(acc, p, nullptr, h, r);
  }
  gejr pj;
  pj.x = p.x;
  pj.y = p.y;
  pj.z = fr_one();
  s = gejr_select(inf, pj, s);
  acc = gejr_select(use, s, acc);
  inf = use ? (inf ? false : to_inf) : inf;
}

// split form: SPLIT_W0 signed RBITS-bit windows, then (carry included) HWIN signed HBITS-bit ones,
// so that h = sum lo_w 2^(RBITS w) + 2^(RBITS SPLIT_W0) sum hi_w 2^(HBITS w)
template <int W>
DEV void recode_step(uint32_t m[5], int& carry, bool neg, int8_t& out) {
  int v = (int)(m[0] & ((1u << W) - 1)) + carry;
  carry = v > (1 << (W - 1)) ? 1 : 0;
  v -= carry << W;
  out = (int8_t)(neg ? -v : v);  // every lane writes the same value
#pragma unroll
  for (int i = 0; i < 4; ++i) m[i] = (m[i] >> W) | (m[i + 1] << (32 - W));
  m[4] >>= W;
}
template <int W0, int NH>
DEV void recode_split(const glv_half& h, int8_t* lo, int8_t* hi) {
  uint32_t m[5];
#pragma unroll
  for (int i = 0; i < 5; ++i) m[i] = h.mag[i];
  int carry = 0;
#pragma unroll 1
  for (int w = 0; w < W0; ++w) recode_step<RBITS>(m, carry, h.neg, lo[w]);
#pragma unroll 1
  for (int w = 0; w < NH; ++w) recode_step<HBITS>(m, carry, h.neg, hi[w]);
}

// GLV split of u_r into signed 5-bit windows (core.cuh ecmult_core's digits; the split and
// three-wave forms' high parts in 4-bit ones), u_g for the comb
template <int FORM>
DEV void recode_r(const sc& u_r, LatLds& S) {
  glv_half h1, h2;
  glv_split(h1, h2, u_r);
  if (FORM == FORM_SPLIT) {
    recode_split<SPLIT_W0, HWIN>(h1, S.rdig[0], S.hdig[0]);
    recode_split<SPLIT_W0, HWIN>(h2, S.rdig[1], S.hdig[1]);
  } else if (FORM == FORM_TRI) {
    recode_split<TRI_W0, TRI_HWIN>(h1, S.rdig[0], S.hdig[0]);
    recode_split<TRI_W0, TRI_HWIN>(h2, S.rdig[1], S.hdig[1]);
  } else {
    recode_row<RBITS, RWIN, int8_t>(h1, S.rdig[0]);
    recode_row<RBITS, RWIN, int8_t>(h2, S.rdig[1]);
  }
}
// u_g in unsigned 16-bit digits for the comb (every lane writes the same values)
DEV void recode_g(const sc& u_g, LatLds& S) {
#pragma unroll
  for (int k = 0; k < CWIN; ++k) S.cdig[k] = (uint16_t)(u_g.v[k >> 1] >> (16 * (k & 1)));
}

// ---- wire form (RecoverParams::wire_*): the transaction's encoding instead of record rows.
// Item idx's bytes [a, e) relative to wire_raw.
DEV bool wire_span(const RecoverParams& prm, uint32_t idx, uint64_t& ra, uint64_t& len) {
  const uint64_t base = prm.wire_off[0], a = prm.wire_off[prm.wire_first + idx], e = prm.wire_off[prm.wire_first + idx + 1];
  const bool ok = e >= a && a >= base;
  ra = ok ? a - base : 0;
  len = ok ? e - a : 0;
  return ok;
}
// The signing hash of m across the wave (keccak_wave.cuh, as tx_rows_wave_kernel), as z mod n;
// zeros for an undecodable item. Optionally written out (lanes 0..3, 8 bytes each).
DEV sc wire_sighash_wave(const Payload& m, bool decoded, uint8_t* out32) {
  const uint32_t lane = lane_id();
  uint64_t st = 0;
  if (decoded) {
    const uint64_t M = m.length();
    const uint64_t nblk = M / 136 + 1;
#pragma unroll 1
    for (uint64_t b = 0; b < nblk; ++b) {
      if (lane < 17) {
        uint64_t x = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const uint64_t j = b * 136 + 8 * lane + k;
          uint64_t byte = j < M ? m.at(j) : 0u;
          if (j == M) byte ^= 0x01u;
          if (b + 1 == nblk && 8 * lane + k == 135) byte ^= 0x80u;
          x |= byte << (8 * k);
        }
        st ^= x;
      }
      keccak_f1600_wave(st);
    }
  }
  if (out32 && lane < 4) {
#pragma unroll
    for (int k = 0; k < 8; ++k) out32[8 * lane + k] = (uint8_t)(st >> (8 * k));
  }
  uint8_t h[32];
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)st, w, 64), hi = (uint32_t)__shfl((int)(uint32_t)(st >> 32), w, 64);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      h[8 * w + k] = (uint8_t)(lo >> (8 * k));
      h[8 * w + 4 + k] = (uint8_t)(hi >> (8 * k));
    }
  }
  uint32_t zl[8];
  limbs_from_be32(zl, h);
  bool ovz;
  return sc_from_limbs(zl, ovz);  // msg mod n (main_impl.h:183)
}

template <int NT>
using TabT = uint32_t[NT][2][16];
template <int NT>
using ColT = uint32_t[NT][16];

// table {1..PTAB} * P on one global Z (co-Z additions, backward rescale; core.cuh); returns zeta.
// P may be the (X, Y) of a Jacobian point: the formulas do not involve the curve's b, so the
// entries are then points of the curve y^2 = x^3 + b Z^6 on which (X, Y) is affine.
template <int NT>
DEV fr build_table_wave(const ger& P, TabT<NT>& tab, ColT<NT>& zrs, ColT<NT>& zq2) {
  static_assert(NT >= 3, "co-Z chain");
  const uint32_t L = row_lane();
  lds_put_pt(tab[0], P);
  gejr D;
  ger B;
  gejq_dblu(D, B, P);
  zrs[0][L] = D.z.v;  // Z_2 / Z_1 = 2y
  ger T;
  T.x = D.x;
  T.y = D.y;
  lds_put_pt(tab[1], T);
  // co-Z additions T += B (gejq_zaddu's values), two quad levels each: the level that forms
  // E = B.y (C - B.x') and T.y also squares the next step's dx = T.x' - B.x', and the next
  // step's dy^2 shares a level with its B.x A, T.x A products. The spare rows square every Z
  // ratio (zq2) and run the product of all of them (zeta, the table's global Z).
  fr dx = fr_normalize_weak(fr_sub<1>(T.x, B.x));
  fr dy = fr_normalize_weak(fr_sub<1>(T.y, B.y));
  fr A, dy2, Bn, C, q, zp;
  fr_mul3(A, dy2, q, dx, dx, dy, dy, D.z, D.z);
  zq2[0][L] = q.v;
  fr_mul3(Bn, C, zp, B.x, A, T.x, A, D.z, dx);
#pragma unroll 1
  for (int i = 2; i < NT; ++i) {  // T = (i+1) P; this step's Z ratio is dx
    const fr tx = fr_normalize_weak(fr_sub<2>(dy2, fr_add(Bn, C)));
    const fr dxn = fr_normalize_weak(fr_sub<1>(tx, Bn));
    fr E, Pd, An;
    fr_mul4(E, Pd, An, q, B.y, fr_sub<1>(C, Bn), dy, fr_sub<1>(Bn, tx), dxn, dxn, dx, dx);
    T.x = tx;
    T.y = fr_normalize_weak(fr_sub<1>(Pd, E));  // dy (B.x' - T.x') - E
    B.x = Bn;
    B.y = E;
    lds_put_pt(tab[i], T);
    zrs[i - 1][L] = dx.v;
    zq2[i - 1][L] = q.v;
    if (i == NT - 1) break;
    dx = dxn;
    dy = fr_normalize_weak(fr_sub<1>(T.y, B.y));
    A = An;
    fr_mul4(dy2, Bn, C, zp, dy, dy, B.x, A, T.x, A, zp, dx);
  }
  // entry i (< NT - 1) is rescaled by rho_i = prod_{k=i}^{NT-2} Z_{k+2}/Z_{k+1} = Z_NT / Z_{i+1}:
  // x rho^2, y rho^3. The cubes of the ratios first (four per quad step, over zrs), then one
  // quad step per entry: x rho_i^2, y rho_i^3, rho_(i-1)^2 = rho_i^2 z^2, rho_(i-1)^3 = rho_i^3 z^3.
#pragma unroll 1
  for (int k = 0; k < NT - 1; k += 4) {
    const int k1 = k + 1 < NT - 1 ? k + 1 : k, k2 = k + 2 < NT - 1 ? k + 2 : k, k3 = k + 3 < NT - 1 ? k + 3 : k;
    fr c0, c1, c2, c3;
    fr_mul4(c0, c1, c2, c3, fr{zrs[k][L]}, fr{zq2[k][L]}, fr{zrs[k1][L]}, fr{zq2[k1][L]}, fr{zrs[k2][L]},
            fr{zq2[k2][L]}, fr{zrs[k3][L]}, fr{zq2[k3][L]});
    zrs[k][L] = c0.v;
    zrs[k1][L] = c1.v;
    zrs[k2][L] = c2.v;
    zrs[k3][L] = c3.v;
  }
  fr s2{zq2[NT - 2][L]}, s3{zrs[NT - 2][L]};
#pragma unroll 1
  for (int i = NT - 2; i >= 0; --i) {
    const ger J = lds_pt(tab[i]);
    const int n = i > 0 ? i - 1 : 0;
    fr ax, ay, s2n, s3n;
    fr_mul4(ax, ay, s2n, s3n, J.x, s2, J.y, s3, s2, fr{zq2[n][L]}, s3, fr{zrs[n][L]});
    ger a;
    a.x = ax;
    a.y = ay;
    lds_put_pt(tab[i], a);
    s2 = s2n;
    s3 = s3n;
  }
  return zp;  // rho_0 = Z_NT / Z_1 with Z_1 = 1
}

// ---- Strauss parts. R' = (c x, c^2) lives on E': y^2 = x^3 + 7 c^3 with c = x^3 + 7 (the image
// of R = (x, y) under the isomorphism (x, y) -> (y^2 x, y^3 y), which needs no square root); the
// R' table on E''s isomorphic curve with global Z = zeta; the G comb on the true curve.

// Windows [wlo, whi) of the GLV halves selected by jmask (bit 0: R digits against tab, bit 1:
// lambda R digits against (btab, tab.y)), Horner from the top window: 5 doublings per window and
// one addition per selected half. The narrow form runs [0, RWIN) with both halves.
template <bool CHECKED, int BITS, int NT>
DEV void strauss_win(gejr& acc, bool& inf, const TabT<NT>& tab, const ColT<NT>& btab, const int8_t* d0,
                     const int8_t* d1, int jmask, int wlo, int whi, const Diag& dg) {
  inf = true;
  acc.x = fr_zero();
  acc.y = fr_zero();
  acc.z = fr_zero();
#pragma unroll 1
  for (int w = whi - 1; w >= wlo; --w) {
    if (w != whi - 1) {
#pragma unroll 1
      for (int k = 0; k < BITS; ++k) acc = gejq_double(acc);
    }
#pragma unroll 1
    for (int j = 0; j < 2; ++j) {
      if (!((jmask >> j) & 1)) continue;
      const int d = (int)(j ? d1 : d0)[w];
      const int a = d < 0 ? -d : d;
      const int e = a > 0 ? a - 1 : 0;
      ger p = lds_pt(tab[e]);
      if (j == 1) p.x.v = btab[e][row_lane()];  // lambda (x, y) = (beta x, y)
      add_r<CHECKED>(acc, inf, ger_neg_if(p, d < 0), d != 0, dg);
    }
  }
}
// window point +-T[|d| - 1] of half j (j = 1: lambda, (beta x, y)); d != 0
template <int NT>
DEV ger win_point(const TabT<NT>& tab, const ColT<NT>& btab, int d, int j) {
  const int e = (d < 0 ? -d : d) - 1;
  ger p = lds_pt(tab[e]);
  if (j == 1) p.x.v = btab[e][row_lane()];
  return ger_neg_if(p, d < 0);
}
// strauss_win<false>'s sums with hoisted additions (frg.cuh gejq_double_pre / gejq_add_pre): each
// window's last doubling starts its first addition and that addition starts the second, so a
// window of BITS doublings and two additions is 3 BITS + 6 quad levels instead of 3 BITS + 10.
// Zero digits are skipped (wave-uniform); windows that start at infinity (the top one, or while
// every digit so far was zero) take the plain steps.
template <int BITS, int NT>
DEV void strauss_win_fast(gejr& acc, bool& inf, const TabT<NT>& tab, const ColT<NT>& btab, const int8_t* d0,
                          const int8_t* d1, int jmask, int wlo, int whi, const Diag& dg) {
  inf = true;
  acc.x = fr_zero();
  acc.y = fr_zero();
  acc.z = fr_zero();
#pragma unroll 1
  for (int w = whi - 1; w >= wlo; --w) {
    const int da = (jmask & 1) ? (int)d0[w] : 0;
    const int db = (jmask & 2) ? (int)d1[w] : 0;
    if (inf) {
      if (w != whi - 1) {
#pragma unroll 1
        for (int k = 0; k < BITS; ++k) acc = gejq_double(acc);
      }
      if (da) add_r<false>(acc, inf, win_point(tab, btab, da, 0), true, dg);
      if (db) add_r<false>(acc, inf, win_point(tab, btab, db, 1), true, dg);
      continue;
    }
    acc = gejq_double_n(acc, BITS - 1);
    if (!da && !db) {
      acc = gejq_double(acc);
      continue;
    }
    const ger first = da ? win_point(tab, btab, da, 0) : win_point(tab, btab, db, 1);
    AddPre pre;
    acc = gejq_double_pre(acc, first.x, pre);
    if (da && db) {
      const ger second = win_point(tab, btab, db, 1);
      AddPre pre2;
      acc = gejq_add_pre<true>(acc, first, pre, second.x, pre2);
      acc = gejq_add_pre<false>(acc, second, pre2, second.x, pre2);
    } else {
      acc = gejq_add_pre<false>(acc, first, pre, first.x, pre);
    }
  }
}
template <int BITS, int NT>
DEV void strauss_win_exact(gejr& acc, bool& inf, const TabT<NT>& tab, const ColT<NT>& btab, const int8_t* d0,
                           const int8_t* d1, int jmask, int wlo, int whi, const Diag& dg) {
  strauss_win_fast<BITS, NT>(acc, inf, tab, btab, d0, d1, jmask, wlo, whi, dg);
  if (dg.force || __any(!inf && fr_is_zero(acc.z))) {
    diag_bump(dg, EGES_DIAG_LAT_REDO);
    strauss_win<true, BITS, NT>(acc, inf, tab, btab, d0, d1, jmask, wlo, whi, dg);
  }
}
// u_g G from the comb table: one addition per 16-bit digit, no doublings (true curve).
template <bool CHECKED>
DEV void strauss_gcomb(gejr& acc, bool& inf, const LatLds& S, const uint32_t* gcomb, const Diag& dg) {
  inf = true;
  acc.x = fr_zero();
  acc.y = fr_zero();
  acc.z = fr_zero();
#pragma unroll 1
  for (int k = 0; k < CWIN; ++k) {
    const int d = (int)S.cdig[k];
    const ger p = gtab_pt(gcomb + ((size_t)k * CTAB + (d > 0 ? d - 1 : 0)) * PT_WORDS);
    add_r<CHECKED>(acc, inf, p, d != 0, dg);
  }
}
// strauss_gcomb<false>'s sum with hoisted additions (frg.cuh gejq_add_pre): the first nonzero
// digit's point starts the sum, every later addition is 3 quad levels and starts the next one.
DEV ger gcomb_pt(const uint32_t* gcomb, int k, int d) {
  return gtab_pt(gcomb + ((size_t)k * CTAB + (d > 0 ? d - 1 : 0)) * PT_WORDS);
}
DEV void strauss_gcomb_fast(gejr& acc, bool& inf, const LatLds& S, const uint32_t* gcomb) {
  int k = 0;
  while (k < CWIN && S.cdig[k] == 0) ++k;
  inf = k == CWIN;
  acc.x = fr_zero();
  acc.y = fr_zero();
  acc.z = fr_zero();
  if (inf) return;
  const ger p0 = gcomb_pt(gcomb, k, S.cdig[k]);
  acc.x = p0.x;
  acc.y = p0.y;
  acc.z = fr_one();
  int kn = k + 1;
  while (kn < CWIN && S.cdig[kn] == 0) ++kn;
  if (kn == CWIN) return;
  ger p = gcomb_pt(gcomb, kn, S.cdig[kn]);
  AddPre pre;  // acc is affine: H = x2 - X1, Z1^3 = 1
  pre.h = fr_normalize_weak(fr_sub<1>(p.x, acc.x));
  pre.z13 = fr_one();
#pragma unroll 1
  for (;;) {
    int kk = kn + 1;
    while (kk < CWIN && S.cdig[kk] == 0) ++kk;
    if (kk == CWIN) {
      acc = gejq_add_pre<false>(acc, p, pre, p.x, pre);
      return;
    }
    const ger q = gcomb_pt(gcomb, kk, S.cdig[kk]);
    AddPre nxt;
    acc = gejq_add_pre<true>(acc, p, pre, q.x, nxt);
    p = q;
    pre = nxt;
    kn = kk;
  }
}
// u_g G, unchecked, with the exact redo (every digit is nonzero-checked, so a poisoned sum
// shows as Z == 0 and not infinity)
DEV void gcomb_exact(gejr& A, bool& ainf, const LatLds& S, const uint32_t* gcomb, const Diag& dg) {
  strauss_gcomb_fast(A, ainf, S, gcomb);
  if (dg.force || __any(!ainf && fr_is_zero(A.z))) {
    diag_bump(dg, EGES_DIAG_COMB_REDO);
    strauss_gcomb<true>(A, ainf, S, gcomb, dg);
  }
}
// exact join of two partial sums, the exceptional branch counted
DEV gejr join_parts(const gejr& a, bool ainf, const gejr& b, bool binf, bool& rinf, const Diag& dg) {
  int exc;
  const gejr r = gejq_add(a, ainf, b, binf, rinf, &exc);
  if (exc) diag_bump(dg, exc == 1 ? EGES_DIAG_JOIN_DBL : EGES_DIAG_JOIN_INF);
  return r;
}
DEV void put_part(LatLds& S, int k, const gejr& a, bool inf) {
  const uint32_t L = row_lane();
  S.part[k][0][L] = a.x.v;
  S.part[k][1][L] = a.y.v;
  S.part[k][2][L] = a.z.v;
  if (lane_id() == 0) S.pinf[k] = inf ? 1u : 0u;
}
DEV gejr get_part(const LatLds& S, int k, bool& inf) {
  const uint32_t L = row_lane();
  gejr a;
  a.x.v = S.part[k][0][L];
  a.y.v = S.part[k][1][L];
  a.z.v = S.part[k][2][L];
  inf = S.pinf[k] != 0;
  return a;
}
// beta x of the 16 table entries, four per quad step
template <int NT>
DEV void build_btab(const TabT<NT>& tab, ColT<NT>& btab) {
  const fr beta = fe_to_fr(fe_const(FE_BETA));
  const uint32_t L = row_lane();
#pragma unroll 1
  for (int i = 0; i < NT; i += 4) {
    fr b0, b1, b2, b3;
    fr_mul4(b0, b1, b2, b3, lds_pt(tab[i]).x, beta, lds_pt(tab[i + 1]).x, beta, lds_pt(tab[i + 2]).x, beta,
            lds_pt(tab[i + 3]).x, beta);
    btab[i][L] = b0.v;
    btab[i + 1][L] = b1.v;
    btab[i + 2][L] = b2.v;
    btab[i + 3][L] = b3.v;
  }
}
// c = x^3 + 7 (magnitude 1)
DEV fr curve_rhs(const fr& x) { return fr_add(fr_mul(fr_sqr(x), x), fr_small(7)); }
// y with y^2 = c and the requested parity (ge_set_xo_var's root); false for a non-residue
DEV bool lift_y(fr& y, const fr& c, bool odd) {
  const bool ok = fr_sqrt(y, c);
  fe yl = fe_normalize(fr_to_fe(y));
  const bool flip = ((yl.v[0] & 1u) != 0) != odd;
  yl = fe_select(flip, fe_normalize(fe_neg<1>(yl)), yl);
  y = fe_to_fr(yl);
  return ok;
}

// Narrow form, wave 1 after the barrier: the square root (when the point came compressed) and
// the u_g G comb part into LDS, then the second barrier. Both run beside wave 0's Strauss loop.
DEV void helper_wave(LatLds& S, const uint32_t* gcomb, bool need_y, const fr& c, bool odd, const fr& y_given,
                     const Diag& dg) {
  fr y = y_given;
  bool ok = true;
  if (need_y) ok = lift_y(y, c, odd);
  S.ylift[row_lane()] = y.v;
  if (lane_id() == 0) S.yok = ok ? 1u : 0u;
  gejr A;
  bool ainf;
  gcomb_exact(A, ainf, S, gcomb, dg);
  put_part(S, 2, A, ainf);
  __syncthreads();  // partial sums and y ready
}
// Split form, wave 1 after its scalar work: y (the square root, or the given y), then u_g G.
DEV void helper_split(LatLds& S, const uint32_t* gcomb, bool need_y, const fr& c, bool odd, const fr& y_given,
                      const Diag& dg) {
  fr y = y_given;
  bool ok = true;
  if (need_y) ok = lift_y(y, c, odd);
  S.ylift[row_lane()] = y.v;
  if (lane_id() == 0) S.yok = ok ? 1u : 0u;
  flag_set(S, F_Y);
  gejr A;
  bool ainf;
  gcomb_exact(A, ainf, S, gcomb, dg);
  put_part(S, 2, A, ainf);
  flag_set(S, F_G);
}
// Split form, waves 2 (j = 0: R) and 3 (j = 1: lambda R): D = 2^(RBITS SPLIT_W0) R' by doublings
// (each wave its own copy, no hand-off), the table of D's (X, Y) on the curve where it is affine,
// the high windows of one GLV half, then back to the true curve: a sum (X, Y, Z) there is the E'
// point (X, Y, Z zeta_D Z_D) and the E point (X, Y, Z zeta_D Z_D y). Wave 2 joins wave 3's part.
DEV void high_wave(LatLds& S, const fr& x, const fr& c, int j, const Diag& dg) {
  gejr D;
  fr_mul2(D.x, D.y, c, x, c, c);  // R' = (c x, c^2)
  D.z = fr_one();
  D = gejq_double_n(D, RBITS * SPLIT_W0);  // R' has odd order: never exceptional
  ger Dp;
  Dp.x = D.x;
  Dp.y = D.y;
  const fr zd = build_table_wave<HTAB>(Dp, S.dtab[j], S.dzr[j], S.dzq[j]);
  if (j == 1) build_btab<HTAB>(S.dtab[1], S.dbtab);
  const fr scale = fr_mul(zd, D.z);
  flag_wait(S, F_DIG);
  gejr A;
  bool ainf;
  strauss_win_exact<HBITS, HTAB>(A, ainf, S.dtab[j], S.dbtab, S.hdig[0], S.hdig[1], 1 << j, 0, HWIN, dg);
  flag_wait(S, F_Y);
  A.z = fr_mul(A.z, fr_mul(scale, fr{S.ylift[row_lane()]}));
  if (j == 1) {
    put_part(S, 4, A, ainf);
    flag_set(S, F_LHI);
    return;
  }
  flag_wait(S, F_LHI);
  bool linf;
  const gejr Lp = get_part(S, 4, linf);
  A = join_parts(A, ainf, Lp, linf, ainf, dg);
  put_part(S, 3, A, ainf);
  flag_set(S, F_HI);
}
// Three-wave form, wave 1 after its scalar work: u_g G (y comes from the root helpers)
DEV void helper_tri(LatLds& S, const uint32_t* gcomb, const Diag& dg) {
  gejr A;
  bool ainf;
  gcomb_exact(A, ainf, S, gcomb, dg);
  put_part(S, 2, A, ainf);
  flag_set(S, F_G);
}
// Three-wave form, wave 2: D = 2^(RBITS TRI_W0) R', D's table and its beta x, the high windows
// of both GLV halves jointly; the sum is published as the E' point (X, Y, Z zeta_D Z_D) (wave 0
// joins it on E' and maps the total to E with y once).
DEV void high_wave_tri(LatLds& S, const fr& x, const fr& c, const Diag& dg) {
  gejr D;
  fr_mul2(D.x, D.y, c, x, c, c);  // R' = (c x, c^2)
  D.z = fr_one();
  D = gejq_double_n(D, RBITS * TRI_W0);  // R' has odd order: never exceptional
  ger Dp;
  Dp.x = D.x;
  Dp.y = D.y;
  const fr zd = build_table_wave<HTAB>(Dp, S.dtab[0], S.dzr[0], S.dzq[0]);
  build_btab<HTAB>(S.dtab[0], S.dbtab);
  const fr scale = fr_mul(zd, D.z);
  flag_wait(S, F_DIG);
  gejr A;
  bool ainf;
  strauss_win_exact<HBITS, HTAB>(A, ainf, S.dtab[0], S.dbtab, S.hdig[0], S.hdig[1], 3, 0, TRI_HWIN, dg);
  A.z = fr_mul(A.z, scale);
  put_part(S, 3, A, ainf);
  flag_set(S, F_HI);
}

// Wave 0: u_r * (x, y) + u_g G with y deferred. R' = (c x, c^2) on E', its table, the digits,
// the R' Strauss sum(s), then back to the true curve: an E' Jacobian point (X, Y, Z) is (X, Y, Z y)
// on E, and the table's isomorphic curve adds the factor zeta. y comes from LDS (helper wave).
// Narrow: both GLV halves over every window here, two barriers. Split: the low windows of both
// halves here; the high windows' sum (waves 2, 3) and u_g G (wave 1) are joined at the end.
DEV void root_fetch(const RecoverParams& prm, uint32_t idx, const fr& c, bool odd, uint32_t epoch, LatLds& S);  // below
struct RootSrc {  // narrow recover form: where wave 0 finds R's y (root_fetch)
  const RecoverParams* prm;
  uint32_t idx;
  bool odd;
  uint32_t epoch;  // the launch's (or the resident server's job's) root-word tag
};
template <class ST, int FORM>
DEV void ecmult_deferred(gejr& Q, bool& qinf, const fr& x, const fr& c, LatLds& S, ST* st, const Diag& dg,
                         const RootSrc* root = nullptr) {
  constexpr bool SPLIT = FORM == FORM_SPLIT;
  ger Rp;
  fr_mul2(Rp.x, Rp.y, c, x, c, c);  // (c x, c^2)
  const fr zeta = build_table_wave<PTAB>(Rp, S.tab, S.zr, S.zq);
  build_btab<PTAB>(S.tab, S.btab);
  st->mark(3);
  if (FORM != FORM_NARROW) flag_wait(S, F_DIG);
  else __syncthreads();  // digits ready
  st->mark(1);
  gejr A;
  bool ainf;
  strauss_win_exact<RBITS, PTAB>(A, ainf, S.tab, S.btab, S.rdig[0], S.rdig[1], 3, 0,
                                 SPLIT ? SPLIT_W0 : FORM == FORM_TRI ? TRI_W0 : RWIN, dg);
  if constexpr (FORM == FORM_TRI) {
    // the low and high sums joined on E' (the addition formulas do not involve b), then to E
    // with y (from the root helpers) once, then + u_g G
    A.z = fr_mul(A.z, zeta);
    flag_wait(S, F_HI);
    bool hinf;
    const gejr Hp = get_part(S, 3, hinf);
    A = join_parts(A, ainf, Hp, hinf, ainf, dg);
    root_fetch(*root->prm, root->idx, c, root->odd, root->epoch, S);
    A.z = fr_mul(A.z, fr{S.ylift[row_lane()]});
    flag_wait(S, F_G);
    bool ginf;
    const gejr Gp = get_part(S, 2, ginf);
    Q = join_parts(A, ainf, Gp, ginf, qinf, dg);
    st->mark(4);
    return;
  }
  if (SPLIT) flag_wait(S, F_Y);
  else __syncthreads();  // partial sums (and y) ready
  if (root) root_fetch(*root->prm, root->idx, c, root->odd, root->epoch, S);  // (this wave's own LDS words)
  A.z = fr_mul(A.z, fr_mul(zeta, fr{S.ylift[row_lane()]}));  // the true curve
  bool ginf;
  if (SPLIT) flag_wait(S, F_G);
  const gejr Gp = get_part(S, 2, ginf);
  Q = join_parts(A, ainf, Gp, ginf, qinf, dg);
  if (SPLIT) {
    flag_wait(S, F_HI);
    bool hinf;
    const gejr Hp = get_part(S, 3, hinf);
    Q = join_parts(Q, qinf, Hp, hinf, qinf, dg);
  }
  st->mark(4);
}

// ---- R's y for the narrow form, lane-serially in helper workgroups.
// At block sizes (n = 1000) two waves share every SIMD and the kernel is bound by total issue;
// wave 1's row-form square root (253 dependent squarings, one row of four busy) was a fifth of
// it. Instead the launch's first ceil(n / 128) workgroups give every signature one lane of a
// lane-serial root (ge_set_xo, ge.cuh) and publish y in the slot rows (unused by this kernel):
// words 0..7 y, 8 ok, 9 epoch tag, 10 ready tag (release, agent scope: readers may sit on
// another XCD). Wave 0 reads it after its Strauss loop; if it is not there within a bound, wave 0
// computes the root itself, so the result never depends on the helpers being scheduled.
constexpr uint32_t ROOT_TAG = 0x9E3779B9u, ROOT_TAG2 = 0x7F4A7C15u;
constexpr int ROOT_WORDS = 11;
static_assert(ROOT_WORDS <= SLOT_ROWS * 4, "the root words live in the slot rows");
constexpr int ROOT_WG = LAT_WG;  // helper lanes per workgroup (same block size as the kernel)
DEV uint32_t* root_area(const RecoverParams& prm) {
  return const_cast<uint32_t*>(prm.rec) + (size_t)REC_ROWS * prm.n_pad;
}

DEV void root_helper(const RecoverParams& prm, uint32_t epoch, uint32_t n) {
  // (the three-wave form's workgroups have 192 threads: the third wave of a helper workgroup
  // would take the next helper's items)
  if (threadIdx.x >= ROOT_WG) return;
  const uint32_t j = blockIdx.x * ROOT_WG + threadIdx.x;
  if (j >= n) return;
  LatParse q;
  if (prm.wire_raw) {  // wire form: this lane decodes item j itself (x, recid, ok: the waves' record)
    uint64_t ra, len;
    const bool sp = wire_span(prm, j, ra, len);
    // Touch every 64-byte line of the encoding first with independent byte loads, so the bytes
    // cross the bus in one round trip (host-memory callers) instead of one per RLP head of the
    // decode below, which then reads them from L2.
    if (sp && len) {
      uint32_t t = 0;
#pragma unroll 1
      for (uint64_t o = ra; o < ra + len; o = (o | 63u) + 1u) t ^= prm.wire_raw[o];
      asm volatile("" ::"v"(t));
    }
    Payload m;
    wire_item(prm.wire_raw + ra, len, sp, prm.wire_signer, prm.wire_chain_id, q, m);
  } else {
    q = prm.snd_r ? sender_parse_lane(prm, j) : lat_parse(prm, j);
  }
  const ge G = gen_point();
  const fe x = q.ok ? fe_from_u256(q.xr) : G.x;  // the row-form waves use the same substitute
  ge r;
  const bool ok = ge_set_xo(r, x, q.ok && (q.recid & 1u) != 0);
  uint32_t y[8];
  fe_to_u256(y, r.y);
  uint32_t* a = root_area(prm);
  const size_t np = prm.n_pad;
#pragma unroll
  for (int i = 0; i < 8; ++i) a[i * np + j] = y[i];
  a[8 * np + j] = ok ? 1u : 0u;
  a[9 * np + j] = epoch ^ ROOT_TAG2;
  __hip_atomic_store(&a[10 * np + j], epoch ^ ROOT_TAG, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}

// wave 0 of signature idx: y and ok into LDS, from the helpers or (bounded wait) computed here
DEV void root_fetch(const RecoverParams& prm, uint32_t idx, const fr& c, bool odd, uint32_t epoch, LatLds& S) {
  uint32_t* a = root_area(prm);
  const size_t np = prm.n_pad;
  bool got = false;
#pragma unroll 1
  for (int it = 0; it < 40000; ++it) {  // ~4 ms: the helpers normally finish long before
    if (__hip_atomic_load(&a[10 * np + idx], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == (epoch ^ ROOT_TAG) &&
        __hip_atomic_load(&a[9 * np + idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (epoch ^ ROOT_TAG2)) {
      got = true;
      break;
    }
    __builtin_amdgcn_s_sleep(4);
  }
  fr y;
  bool ok;
  if (got) {
    uint32_t w[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) w[i] = __hip_atomic_load(&a[i * np + idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    y = fe_to_fr(fe_from_u256(w));
    ok = __hip_atomic_load(&a[8 * np + idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
  } else {
    ok = lift_y(y, c, odd);
  }
  S.ylift[row_lane()] = y.v;
  if (lane_id() == 0) S.yok = ok ? 1u : 0u;
}

// diagnostic build: where this wave runs, XCC_ID << 16 | HW_ID[15:0] (wave slot, SIMD, CU, SH, SE)
DEV uint32_t hw_place() {
  uint32_t hw, xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  return (xcc & 0xfu) << 16 | (hw & 0xffffu);
}

// Phase marks of wave 0 (diagnostic build only): 0 parse + x, c, 3 table, 1 wait for wave 1's
// r^-1 / u1 / u2 / digits, 4 Strauss + join (including the waits for the other parts and y),
// 5 Z^-1 + affine, 6 Keccak + stores.
// Narrow form (two waves): wave 0 table + both GLV halves; wave 1 the scalar work, then the
// square root and the u1 G comb part. SPLIT (small batches, four waves): wave 1 the scalar work,
// y and u1 G; waves 2 and 3 the high windows of the two GLV halves against their own table of
// D = 2^75 R'; wave 0 the low windows of both halves, then joins the three partial sums.
template <class ST, int FORM>
DEV void recover_lat_item(const RecoverParams& prm, uint32_t idx, LatLds& S, uint64_t* stamps, uint32_t epoch);
template <class ST, int FORM>
DEV void recover_lat_body(const RecoverParams& prm, uint64_t* stamps) {
  constexpr bool SPLIT = FORM == FORM_SPLIT;
  __shared__ LatLds S;
  gate_wait(prm);
  if (!SPLIT && blockIdx.x < prm.n_helpers) {  // narrow / three-wave forms: the lane-serial roots
    root_helper(prm, prm.epoch, prm.n);
    return;
  }
  recover_lat_item<ST, FORM>(prm, blockIdx.x - (SPLIT ? 0u : prm.n_helpers), S, stamps, prm.epoch);  // a signature per workgroup
}
// signature idx on this workgroup (all its waves enter; each returns when its part is done)
template <class ST, int FORM>
DEV void recover_lat_item(const RecoverParams& prm, uint32_t idx, LatLds& S, uint64_t* stamps, uint32_t epoch) {
  constexpr bool SPLIT = FORM == FORM_SPLIT;   // four waves, wave 1 computes y
  constexpr bool FLAGS = FORM != FORM_NARROW;  // LDS flag hand-offs instead of barriers
  ST st_;
  ST* st = &st_;
  const Diag dg = diag_of(prm);
  // the helpers' lane-serial roots are a dense VALU stream: the signature waves (latency-bound
  // chains) take issue priority over them on a shared SIMD
  if (!SPLIT) __builtin_amdgcn_s_setprio(2);
  const bool wire = prm.wire_raw != nullptr;  // kernel-uniform
  uint64_t wra = 0, wlen = 0;
  bool wspan = false;
  if (wire) {  // the encoding into LDS (one byte per thread per step, coalesced)
    wspan = wire_span(prm, idx, wra, wlen);
    if (wlen <= LAT_STAGE)
      for (uint32_t j = threadIdx.x; j < wlen; j += blockDim.x) S.stage[j] = prm.wire_raw[wra + j];
  }
  if (FLAGS && threadIdx.x < NFLAGS) S.flag[threadIdx.x] = 0u;
  if (FLAGS && threadIdx.x == 0) S.skip = idx == prm.test_skip_block ? prm.test_skip_flag : 0u;  // (item index)
  if (FLAGS || wire) __syncthreads();  // (split / three-wave: the only barrier; narrow: the stage)
  // --- parse (every lane reads the same record; wire form: every lane decodes the same item)
  LatParse q;
  Payload m;
  bool decoded = false;
  if (wire) {
    const uint8_t* p = wlen <= LAT_STAGE ? S.stage : prm.wire_raw + wra;
    decoded = wire_item(p, wlen, wspan, prm.wire_signer, prm.wire_chain_id, q, m);
    q.Z = sc_zero();  // (wave 1 hashes m for z)
  } else {
    q = prm.snd_r ? sender_parse_wave(prm, idx) : lat_parse(prm, idx);  // (fused prep_sender / prep)
  }
  const uint32_t meta = q.meta, recid = q.recid;
  bool ok = q.ok;
  sc R = q.R;
  const sc Sv = q.Sv, Z = q.Z;
  uint32_t xr[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) xr[i] = q.xr[i];
  // R's x; signatures that fail the parse carry the generator's x (even y), so every later step
  // stays well-defined. c = x^3 + 7 = y^2 (ge_set_xo_var, group_impl.h:216-237).
  const ge G = gen_point();
  const fr x = fr_select(ok, fe_to_fr(fe_from_u256(xr)), fe_to_fr(G.x));
  const bool odd = ok && (recid & 1u) != 0;
  const fr c = curve_rhs(x);
  const uint32_t* gcomb = prm.gtab + (size_t)2 * GTAB * PT_WORDS;
  const uint32_t wv = threadIdx.x >> 6;
  if (wv == 1) {
    // --- u1 = -z / r, u2 = s / r (main_impl.h:114-117), digits into LDS
    constexpr bool stamped = !std::is_same<ST, NoStamp>::value;
    const uint64_t t0 = stamped ? __builtin_amdgcn_s_memtime() : 0;
    R = sc_select(ok, R, sc_one());
    const sc rinv = sc_inv_row_var(R);  // wave-uniform data: variable-time safegcd, limb-parallel
    const uint64_t t1 = stamped ? __builtin_amdgcn_s_memtime() : 0;
    const sc u2 = sc_select(ok, sc_mul(rinv, Sv), sc_one());
    if (wire) {
      // the R digits first (wave 0 is waiting for them), then the signing hash for z and u1
      recode_r<FORM>(u2, S);
      if (FLAGS) flag_set(S, F_DIG);
      else __syncthreads();  // digits ready (and the table)
      uint8_t* hs = prm.wire_sighash ? prm.wire_sighash + (size_t)idx * 32 : nullptr;
      recode_g(sc_neg(sc_mul(rinv, wire_sighash_wave(m, decoded, hs))), S);
    } else {
      recode_r<FORM>(u2, S);  // the R digits first: wave 0 is waiting for them
      if (FLAGS) flag_set(S, F_DIG);
      else __syncthreads();  // digits ready (and the table)
      recode_g(sc_neg(sc_mul(rinv, Z)), S);  // u1 = -z / r, for this wave's comb
    }
    if (stamped && lane_id() == 0) {
      S.w1t[0] = (t1 - t0) | ((uint64_t)hw_place() << 32);
      S.w1t[1] = __builtin_amdgcn_s_memtime() - t1;
    }
    if (SPLIT) helper_split(S, gcomb, true, c, odd, fr_zero(), dg);
    else if (FORM == FORM_TRI) helper_tri(S, gcomb, dg);  // y: the helper workgroups (root_fetch)
    else helper_wave(S, gcomb, false, c, odd, fr_zero(), dg);
    return;
  }
  if (SPLIT && (wv == 2 || wv == 3)) {
    high_wave(S, x, c, (int)wv - 2, dg);
    return;
  }
  if (FORM == FORM_TRI && wv == 2) {
    if (idx == 0) diag_bump(dg, EGES_DIAG_LAT_TRI);  // (once per launch: tests see the form ran)
    high_wave_tri(S, x, c, dg);
    return;
  }
  st->mark(0);
  // --- Q = u2 R + u1 G, R's y (the square root) computed beside the Strauss loop
  gejr Q;
  bool qinf;
  const RootSrc root{&prm, idx, odd, epoch};
  ecmult_deferred<ST, FORM>(Q, qinf, x, c, S, st, dg, SPLIT ? nullptr : &root);
  const bool fault = FLAGS && ho_failed(&S.flag[F_ERR], dg);  // after wave 0's last wait
  ok = ok && S.yok != 0 && !qinf && !fault;  // ge_set_xo_var failure, main_impl.h:120
  // --- affine, serialize, address
  const fr zq = fr_select(ok, Q.z, fr_one());
  const fr zi = fr_inv_var(zq);  // row-parallel safegcd (modinv_row.cuh)
  fr zi2, zi3;
  zi2 = fr_sqr(zi);
  fr X1, Y1;
  fr_mul2(X1, zi3, Q.x, zi2, zi2, zi);
  Y1 = fr_mul(Q.y, zi3);
  uint32_t X[8], Y[8];
  fe_to_u256(X, fe_normalize(fr_to_fe(X1)));
  fe_to_u256(Y, fe_normalize(fr_to_fe(Y1)));
  st->mark(5);
  uint32_t a[5];
  pub_address_wave(a, X, Y);  // Keccak across the wave's lanes (keccak_wave.cuh)
  if (lane_id() == 0) {
    const uint32_t pre_st = (meta >> 8) & 0xffu;
    const uint32_t stv = fault ? ST_ENGINE_FAULT : pre_st != ST_OK ? pre_st : (ok ? ST_OK : ST_RECOVER_FAILED);
    prm.status[idx] = (uint8_t)stv;
    if (prm.addr) {
      uint32_t* dst = reinterpret_cast<uint32_t*>(prm.addr + (size_t)idx * prm.addr_stride);
#pragma unroll
      for (int i = 0; i < 5; ++i) dst[i] = ok ? a[i] : 0u;
    }
    if (prm.pub) {
      uint8_t* dst = prm.pub + (size_t)idx * 65;
      if (ok) {
        dst[0] = 4;
        write_be32(dst + 1, X);
        write_be32(dst + 33, Y);
      } else {
        for (int i = 0; i < 65; ++i) dst[i] = 0;
      }
    }
    if (prm.out_tag) {  // the resident server (launch.h out_tag_recover): over the bytes just stored
      uint32_t be[16];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        be[j] = (ok && prm.pub) ? X[7 - j] : 0u;
        be[8 + j] = (ok && prm.pub) ? Y[7 - j] : 0u;
      }
      prm.out_tag[idx] = out_tag_recover(prm.tag_seq, stv, (ok && prm.pub) ? 4u : 0u, be);
    }
  }
  st->mark(6);
  if constexpr (!std::is_same<ST, NoStamp>::value) {
    // wave 1's phases in the unused slots (not part of wave 0's total); the high words carry
    // where wave 1 (slot 2) and wave 0 (slot 7) ran (hw_place)
    st_.acc[2] = S.w1t[0];
    st_.acc[7] = S.w1t[1] | ((uint64_t)hw_place() << 32);
    if (lane_id() == 0) {
#pragma unroll
      for (int i = 0; i < 8; ++i) stamps[(size_t)idx * 8 + i] = st_.acc[i];
    }
  }
}

// ------------------------------------------------------------------ verify, one item per wave
// crypto.VerifySignature for small batches (verify_kernel's checks, k_verify.hip; ext.h:58-75,
// eckey_impl.h:17-34, secp256k1.c:293-308, ecdsa_impl.h:203-271): wave 1 computes s^-1
// (variable-time safegcd), u1 = z/s, u2 = r/s and the digits while wave 0 parses the public key
// (the square root for 33-byte keys, the curve equation for 65-byte ones); then Q = u2 P + u1 G
// and x(Q) == r checked projectively (r Z^2 == X), no field inversion.
template <bool SPLIT>
DEV void verify_lat_item(const VerifyParams& prm, uint32_t idx, LatLds& S);
template <bool SPLIT>
DEV void verify_lat_body(const VerifyParams& prm) {
  __shared__ LatLds S;
  verify_lat_item<SPLIT>(prm, blockIdx.x, S);  // grid = n
}
template <bool SPLIT>
DEV void verify_lat_item(const VerifyParams& prm, uint32_t idx, LatLds& S) {
  NoStamp st_;
  const Diag dg = diag_of(prm);
  if (SPLIT) {
    if (threadIdx.x < NFLAGS) S.flag[threadIdx.x] = 0u;
    if (threadIdx.x == 0) S.skip = idx == prm.test_skip_block ? prm.test_skip_flag : 0u;
    __syncthreads();  // the only barrier of the split form
  }
  uint32_t l[8];
  bool ovr, ovs, ovz;
  limbs_from_be32(l, prm.sig + (size_t)idx * 64);
  const sc R = sc_from_limbs(l, ovr);
  limbs_from_be32(l, prm.sig + (size_t)idx * 64 + 32);
  const sc Sv = sc_from_limbs(l, ovs);
  limbs_from_be32(l, prm.msg + (size_t)idx * 32);
  const sc Z = sc_from_limbs(l, ovz);  // the message reduced mod n
  // parse_compact overflow, high s (ecdsa_verify), r or s zero (sig_verify)
  const bool sig_ok = !ovr && !ovs && !sc_is_high(Sv) && !sc_is_zero(R) && !sc_is_zero(Sv);
  // --- public key (eckey_impl.h:17-34)
  const uint32_t plen = prm.publen[idx];
  const uint8_t* pk = prm.pub + (size_t)idx * 65;
  const uint32_t pfx = pk[0];
  uint32_t px[8], py[8];
  limbs_from_be32(px, pk + 1);
  if (plen == 65) {
    limbs_from_be32(py, pk + 33);
  } else {
#pragma unroll
    for (int q = 0; q < 8; ++q) py[q] = 0;
  }
  const bool x_ok = !u256_ge(px, FE_P), y_ok = !u256_ge(py, FE_P);
  const bool c33 = plen == 33 && (pfx == 2 || pfx == 3);
  const bool c65 = plen == 65 && (pfx == 4 || pfx == 6 || pfx == 7);
  const bool hybrid_bad = (pfx == 6 || pfx == 7) && ((py[0] & 1u) != (pfx == 7 ? 1u : 0u));
  // keys that fail the parse carry the generator, so every later step stays well-defined
  const ge G = gen_point();
  const bool use_key = (c33 || c65) && x_ok;
  const fr x = fr_select(use_key, fe_to_fr(fe_from_u256(px)), fe_to_fr(G.x));
  const fr Y = fr_select(use_key && c65, fe_to_fr(fe_from_u256(py)), fe_to_fr(G.y));
  const fr c = curve_rhs(x);
  const uint32_t* gcomb = prm.gtab + (size_t)2 * GTAB * PT_WORDS;
  const uint32_t wv = threadIdx.x >> 6;
  if (wv == 1) {
    const sc sinv = sc_inv_row_var(sc_select(sig_ok, Sv, sc_one()));
    const sc u2 = sc_select(sig_ok, sc_mul(sinv, R), sc_one());
    recode_r<SPLIT ? FORM_SPLIT : FORM_NARROW>(u2, S);  // the key's digits first: wave 0 is waiting for them
    if (SPLIT) flag_set(S, F_DIG);
    else __syncthreads();  // digits ready (and the table)
    recode_g(sc_mul(sinv, Z), S);  // u1 = z / s
    // the square root only for 33-byte keys; 65-byte keys give y
    if (SPLIT) helper_split(S, gcomb, c33, c, pfx == 3, Y, dg);
    else helper_wave(S, gcomb, c33, c, pfx == 3, Y, dg);
    return;
  }
  if (SPLIT && (wv == 2 || wv == 3)) {
    high_wave(S, x, c, (int)wv - 2, dg);
    return;
  }
  const bool on = fr_equal(c, fr_sqr(Y));  // 65-byte keys: on the curve
  gejr Q;
  bool qinf;
  ecmult_deferred<NoStamp, SPLIT ? FORM_SPLIT : FORM_NARROW>(Q, qinf, x, c, S, &st_, dg);
  const bool fault = SPLIT && ho_failed(&S.flag[F_ERR], dg);  // after wave 0's last wait (F_HI)
  const bool pk_ok = c33 ? (x_ok && S.yok != 0) : (c65 && x_ok && y_ok && !hybrid_bad && on);
  bool ok = sig_ok && pk_ok && !qinf;
  // x(Q) mod n == r  <=>  r Z^2 == X  or  (r < p - n and (r + n) Z^2 == X)  (ecdsa_impl.h:246-270)
  const fr z2 = fr_sqr(Q.z);
  bool eq = fr_equal(Q.x, fr_mul(fe_to_fr(fe_from_u256(R.v)), z2));
  if (!eq && !u256_ge(R.v, P_MINUS_N)) {
    uint32_t rn[8];
    uint64_t c = 0;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      c += (uint64_t)R.v[q] + SC_N[q];
      rn[q] = (uint32_t)c;
      c >>= 32;
    }
    eq = fr_equal(Q.x, fr_mul(fe_to_fr(fe_from_u256(rn)), z2));
  }
  if (lane_id() == 0) {  // ok stays 0 / 1 (eges.h): a faulted item reads invalid, the fault word says why
    const uint32_t v = (!fault && ok && eq) ? 1u : 0u;
    prm.ok[idx] = (uint8_t)v;
    if (fault && prm.fault) __hip_atomic_store(prm.fault, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (prm.out_tag) prm.out_tag[idx] = out_tag_verify(prm.tag_seq, v, fault ? 1u : 0u);  // (launch.h)
  }
}

constexpr int LAT_WG_SPLIT = 256;  // split form: four waves

__global__ void __launch_bounds__(LAT_WG) verify_lat_kernel(VerifyParams prm) { verify_lat_body<false>(prm); }
__global__ void __launch_bounds__(LAT_WG_SPLIT) verify_lat_split_kernel(VerifyParams prm) { verify_lat_body<true>(prm); }

hipError_t launch_verify_lat(const VerifyParams& p, bool wide, hipStream_t st) {
  if (p.n == 0) return hipSuccess;
  if (wide) hipLaunchKernelGGL(verify_lat_split_kernel, dim3(p.n), dim3(LAT_WG_SPLIT), 0, st, p);
  else hipLaunchKernelGGL(verify_lat_kernel, dim3(p.n), dim3(LAT_WG), 0, st, p);
  return hipGetLastError();
}

constexpr int LAT_WG_TRI = 192;  // three-wave form
__global__ void __launch_bounds__(LAT_WG) recover_lat_kernel(RecoverParams prm) {
  recover_lat_body<NoStamp, FORM_NARROW>(prm, nullptr);
}
__global__ void __launch_bounds__(LAT_WG_SPLIT) recover_lat_split_kernel(RecoverParams prm) {
  recover_lat_body<NoStamp, FORM_SPLIT>(prm, nullptr);
}
__global__ void __launch_bounds__(LAT_WG_TRI) recover_lat_tri_kernel(RecoverParams prm) {
  recover_lat_body<NoStamp, FORM_TRI>(prm, nullptr);
}

// the narrow and three-wave forms' launch: ceil(n / 128) root-helper workgroups first (dispatched
// before the signatures' workgroups), tagged with a per-launch epoch so stale slot-row words never
// match
static std::atomic<uint32_t> g_root_epoch{0};
static RecoverParams with_helpers(const RecoverParams& p0) {
  RecoverParams p = p0;
  p.n_helpers = p.wide == FORM_SPLIT ? 0u : (p.n + ROOT_WG - 1) / ROOT_WG;
  // tests only: no helper workgroups, so every signature wave takes root_fetch's own-root path
  if (knob(KNOB_ROOT_HELPERS) == 0) p.n_helpers = 0;
  p.epoch = g_root_epoch.fetch_add(1) + 1u;
  return p;
}
hipError_t launch_recover_lat(const RecoverParams& p0, hipStream_t st) {
  if (p0.n == 0) return hipSuccess;
  const RecoverParams p = with_helpers(p0);
  if (p.wide == FORM_SPLIT) hipLaunchKernelGGL(recover_lat_split_kernel, dim3(p.n), dim3(LAT_WG_SPLIT), 0, st, p);
  else if (p.wide == FORM_TRI)
    hipLaunchKernelGGL(recover_lat_tri_kernel, dim3(p.n_helpers + p.n), dim3(LAT_WG_TRI), 0, st, p);
  else hipLaunchKernelGGL(recover_lat_kernel, dim3(p.n_helpers + p.n), dim3(LAT_WG), 0, st, p);
  return hipGetLastError();
}

// ---- resident servers (launch.h ResidentParams). Workgroup 0's thread 0 polls the host's job word
// (system-scope acquire, s_sleep between polls) and mirrors each job into device memory (the
// words after the completion counters); every other workgroup polls the mirror, so the host
// memory sees one poller whatever the grid (a poller per workgroup over PCIe slowed a
// 1,000-workgroup grid tenfold). Workgroup 0 alone decides to exit (the stop word, or idle_ticks
// without a job), so the grid leaves together. Each workgroup takes items blockIdx.x,
// + gridDim.x, ... and counts itself done; the last one stores the job's sequence into `done`
// after every workgroup's outputs (each releases at system scope before its count).
// RM_SEQ: one 64-bit word (launch id << 32 | sequence), so a workgroup never pairs this launch's
// id with an earlier launch's sequence (launch.h RESIDENT_COUNTER_BYTES covers the mirror)
enum { RM_SEQ = 8, RM_EXIT = 10, RM_N, RM_KIND, RM_END };
static_assert(RM_END * 4 <= RESIDENT_COUNTER_BYTES, "resident mirror");
struct ResidentNext {
  uint32_t seq, n, kind, exit;
};
// thread 0: the next job (one the host handed over and no launch has served yet: seq > done)
// after `seen`, or this launch's exit, into J. The mirror entries carry the launch's id, so a
// launch queued behind another never takes the earlier one's mirror for its own.
DEV void resident_next(const ResidentParams& rp, uint32_t seen, uint64_t last, ResidentNext& J) {
  uint32_t* M = rp.counter;
  if (blockIdx.x == 0) {
    uint32_t q = seen, stop = 0;
#pragma unroll 1
    for (;;) {
      q = __hip_atomic_load(&rp.job->seq, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
      stop = __hip_atomic_load(&rp.job->stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      const uint32_t d = __hip_atomic_load(&rp.job->done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      if (stop || (q != seen && q > d)) break;
      if (__builtin_amdgcn_s_memrealtime() - last > rp.idle_ticks) {
        stop = 1;
        break;
      }
      __builtin_amdgcn_s_sleep(8);
    }
    if (stop) {
      J.exit = 1;
      __hip_atomic_store(&M[RM_EXIT], rp.inst, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      return;
    }
    J.exit = 0;
    J.seq = q;
    J.n = __hip_atomic_load(&rp.job->n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    J.kind = __hip_atomic_load(&rp.job->kind, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (gridDim.x > 1) {
      __hip_atomic_store(&M[RM_N], J.n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&M[RM_KIND], J.kind, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(reinterpret_cast<uint64_t*>(M + RM_SEQ), (uint64_t)rp.inst << 32 | q, __ATOMIC_RELEASE,
                         __HIP_MEMORY_SCOPE_AGENT);
    }
    return;
  }
#pragma unroll 1
  for (;;) {
    const uint32_t e = __hip_atomic_load(&M[RM_EXIT], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t qi = __hip_atomic_load(reinterpret_cast<uint64_t*>(M + RM_SEQ), __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t q = (uint32_t)qi, inst = (uint32_t)(qi >> 32);
    if (e == rp.inst) {  // (this launch's exit; earlier launches' marks carry their own ids)
      J.exit = 1;
      return;
    }
    if (inst == rp.inst && q > seen) {
      // the job's inputs sit in cacheable pinned memory the host just wrote: a system-scope
      // acquire (cache invalidation) on this workgroup's side too
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
      J.exit = 0;
      J.seq = q;
      J.n = __hip_atomic_load(&M[RM_N], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      J.kind = __hip_atomic_load(&M[RM_KIND], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return;
    }
    __builtin_amdgcn_s_sleep(8);
  }
}
// thread 0: this workgroup is done with job seq; the last one publishes it. (The host does not
// rely on `done` reaching it after the outputs: each item carries a tag over its output bytes,
// launch.h out_tag_recover / out_tag_verify, which the host checks.)
DEV void resident_done(const ResidentParams& rp, uint32_t seq) {
  if (blockIdx.x == 0 && rp.diag) __hip_atomic_fetch_add(rp.diag + EGES_DIAG_RESIDENT, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // this workgroup's outputs (thread 0 wrote them), system scope
  const uint32_t c = __hip_atomic_fetch_add(&rp.counter[seq & 1u], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
  if (c == gridDim.x - 1) {
    __hip_atomic_store(&rp.counter[seq & 1u], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&rp.job->done, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// The single-call server: coalesced groups of eges_ecdsa_recover / eges_ecdsa_verify (split form).
__global__ void __launch_bounds__(LAT_WG_SPLIT) lat_resident_kernel(ResidentParams rp) {
  __shared__ LatLds S;
  __shared__ ResidentNext J;
  uint32_t seen = rp.seen0;
  uint64_t last = __builtin_amdgcn_s_memrealtime();
#pragma unroll 1
  for (;;) {
    if (threadIdx.x == 0) resident_next(rp, seen, last, J);
    __syncthreads();
    if (J.exit) return;
    const uint32_t seq = J.seq, n = J.n < rp.cap ? J.n : rp.cap, kind = J.kind;
    const ResidentLayout L = resident_layout(rp.cap);
#pragma unroll 1
    for (uint32_t idx = blockIdx.x; idx < n; idx += gridDim.x) {
      if (kind == RESIDENT_RECOVER) {
        RecoverParams p{nullptr, n, n, rp.data + L.status, nullptr, rp.data + L.pub, rp.gtab, nullptr};
        p.raw_msg = rp.data + L.msg;
        p.raw_sig = rp.data + L.sig;
        p.wide = FORM_SPLIT;
        p.diag = rp.diag;
        p.out_tag = reinterpret_cast<uint64_t*>(rp.data + L.tag);
        p.tag_seq = seq;
        recover_lat_item<NoStamp, FORM_SPLIT>(p, idx, S, nullptr, 0u);
      } else {
        VerifyParams v{rp.data + L.vpub, rp.data + L.vpublen, rp.data + L.vmsg, rp.data + L.vsig, n,
                       rp.data + L.vok, rp.gtab, nullptr};
        v.diag = rp.diag;
        v.fault = reinterpret_cast<uint32_t*>(rp.data + L.vfault);
        v.out_tag = reinterpret_cast<uint64_t*>(rp.data + L.tag);
        v.tag_seq = seq;
        verify_lat_item<true>(v, idx, S);
      }
      __syncthreads();  // every wave done with this item's LDS
    }
    if (threadIdx.x == 0) resident_done(rp, seq);
    seen = seq;
    last = __builtin_amdgcn_s_memrealtime();
    __syncthreads();  // (J is rewritten by the next poll)
  }
}
hipError_t launch_lat_resident(const ResidentParams& p, uint32_t wgs, hipStream_t st) {
  hipLaunchKernelGGL(lat_resident_kernel, dim3(wgs), dim3(LAT_WG_SPLIT), 0, st, p);
  return hipGetLastError();
}

#ifdef EGES_PHASE_STAMPS
__global__ void __launch_bounds__(LAT_WG) recover_lat_kernel_stamped(RecoverParams prm, uint64_t* stamps) {
  recover_lat_body<Stamper, FORM_NARROW>(prm, stamps);
}
__global__ void __launch_bounds__(LAT_WG_SPLIT) recover_lat_split_kernel_stamped(RecoverParams prm, uint64_t* stamps) {
  recover_lat_body<Stamper, FORM_SPLIT>(prm, stamps);
}
__global__ void __launch_bounds__(LAT_WG_TRI) recover_lat_tri_kernel_stamped(RecoverParams prm, uint64_t* stamps) {
  recover_lat_body<Stamper, FORM_TRI>(prm, stamps);
}
hipError_t launch_recover_lat_stamped(const RecoverParams& p0, hipStream_t st, uint64_t* stamps) {
  if (p0.n == 0) return hipSuccess;
  const RecoverParams p = with_helpers(p0);
  if (p.wide == FORM_SPLIT)
    hipLaunchKernelGGL(recover_lat_split_kernel_stamped, dim3(p.n), dim3(LAT_WG_SPLIT), 0, st, p, stamps);
  else if (p.wide == FORM_TRI)
    hipLaunchKernelGGL(recover_lat_tri_kernel_stamped, dim3(p.n_helpers + p.n), dim3(LAT_WG_TRI), 0, st, p, stamps);
  else hipLaunchKernelGGL(recover_lat_kernel_stamped, dim3(p.n_helpers + p.n), dim3(LAT_WG), 0, st, p, stamps);
  return hipGetLastError();
}
size_t lat_waves(uint32_t n) { return n; }
#endif

}  // namespace eges
