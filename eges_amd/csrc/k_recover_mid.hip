// Mid-size recover kernel: batches too large for the latency kernels (one signature per wave)
// and too small to fill the GPU lane-serially (one signature per lane, k_recover.hip).
//
// Same path and outputs as recover_kernel (recovery/main_impl.h:38-191, ecmult_impl.h:286-404,
// eckey_impl.h:36-52, crypto.go:194-197). A workgroup takes 64 signatures, one per lane, and
// gives each of its four waves one ROLE of Q = u2 R + u1 G for all 64 (roles are wave-uniform,
// so there is no divergence; every lane works lane-serially on its own signature with the
// radix-2^29 core of fe.cuh, the throughput kernel's arithmetic):
//
//   wave 1 "S"  parse, r^-1 (safegcd), u1 = -z / r, u2 = s / r, GLV split of u2 and the digits
//               (LDS) -> R's y (square root) -> u1 G by the 16-bit comb (true curve)
//   wave 0 "A"  R' = (c x, c^2) on E': y^2 = x^3 + 7 c^3 (c = x^3 + 7; no square root), its
//               16-entry table on one global Z, windows [0, 15) of both GLV halves; then the
//               joins, Z^-1, affine, Keccak address, stores
//   wave 2 "B"  D = 2^75 R' by doublings, an 8-entry table of D, the high windows of the R half
//   wave 3 "C"  the same for the lambda R half
//
// The parts meet through LDS with flags (release fence + flag store, consumers poll), so no wave
// waits for work it does not consume. The critical path is a high wave's ~130 doublings instead
// of a whole signature's chain: a batch of a few thousand to a few tens of thousands of
// signatures finishes in well under the lane-serial kernel's fixed ~0.8 ms.
//
// Exceptional sums: the R-table loops and the comb cannot meet acc == +-P (DESIGN.md §3.1,
// tests/test_exceptional_model.py); they still run unchecked with an exact redo, as the other
// kernels do. The joins are exact additions (a == b doubles, a == -b is infinity).
#include <type_traits>

#include "core.cuh"
#include "handoff.cuh"
#include "modinv_row.cuh"
#include "sender.cuh"

namespace eges {

constexpr int MID_WG = 256;  // four waves
constexpr int MID_L = 64;    // signatures per workgroup (one per lane)
constexpr int MID_W0 = 15;  // windows [0, MID_W0) on wave A, the rest on waves B / C
constexpr int MID_HBITS = 4;
constexpr int MID_HTAB = 1 << (MID_HBITS - 1);
constexpr int MID_HWIN = (130 - RBITS * MID_W0 + MID_HBITS) / MID_HBITS;
static_assert(MID_W0 * RBITS + MID_HWIN * MID_HBITS >= 130, "windows cover a GLV half + carry");

enum { MF_DIG = 0, MF_Y, MF_G, MF_HB, MF_HC, MF_ERR, MF_N };

struct MidLds {
  int8_t lo[2][MID_W0][MID_L];    // 5-bit digits of both halves, windows [0, MID_W0)
  int8_t hi[2][MID_HWIN][MID_L];  // 4-bit digits of the high parts
  uint32_t y[FE_LIMBS][MID_L];    // R's y (wave S)
  uint32_t part[3][3][FE_LIMBS][MID_L];  // 0: u1 G (E), 1 / 2: high parts (E')
  uint32_t pinf[3][MID_L];
  uint32_t yok[MID_L];
  uint32_t flag[MF_N];
};

// Per-workgroup workspace (global memory, L2-resident): the three tables and their Z ratios,
// entry-major then lane (core.cuh layout).
constexpr size_t MID_TAB_A = 0;
constexpr size_t MID_TAB_B = MID_TAB_A + (size_t)PTAB * MID_L * PT_WORDS;
constexpr size_t MID_TAB_C = MID_TAB_B + (size_t)MID_HTAB * MID_L * PT_WORDS;
constexpr size_t MID_ZR_A = MID_TAB_C + (size_t)MID_HTAB * MID_L * PT_WORDS;
constexpr size_t MID_ZR_B = MID_ZR_A + (size_t)(PTAB - 1) * MID_L * ZR_WORDS;
constexpr size_t MID_ZR_C = MID_ZR_B + (size_t)(MID_HTAB - 1) * MID_L * ZR_WORDS;
constexpr size_t MID_WS_WORDS = MID_ZR_C + (size_t)(MID_HTAB - 1) * MID_L * ZR_WORDS;

// Flags between the roles (handoff.cuh): every producer sets its flags unconditionally; the
// bounded waits only keep a logic error from hanging the device or from yielding a result
// computed from unwritten LDS (the output wave then writes ST_ENGINE_FAULT).
#define MFLAG_SET(k) ho_set(&S.flag[k], 1u, ho_skip(prm, k))
#define MFLAG_WAIT(k) ho_wait<2>(&S.flag[k], 1u, &S.flag[MF_ERR])

template <int N>
DEV void lds_put_fe(uint32_t (*a)[MID_L], const uint32_t* v, uint32_t l) {
#pragma unroll
  for (int i = 0; i < N; ++i) a[i][l] = v[i];
}
template <int N>
DEV void lds_get_fe(const uint32_t (*a)[MID_L], uint32_t* v, uint32_t l) {
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] = a[i][l];
}
DEV void put_part_ls(MidLds& S, int k, const gej& p, bool inf, uint32_t l) {
  lds_put_fe<FE_LIMBS>(S.part[k][0], p.x.v, l);
  lds_put_fe<FE_LIMBS>(S.part[k][1], p.y.v, l);
  lds_put_fe<FE_LIMBS>(S.part[k][2], p.z.v, l);
  S.pinf[k][l] = inf ? 1u : 0u;
}
DEV gej get_part_ls(const MidLds& S, int k, bool& inf, uint32_t l) {
  gej p;
  lds_get_fe<FE_LIMBS>(S.part[k][0], p.x.v, l);
  lds_get_fe<FE_LIMBS>(S.part[k][1], p.y.v, l);
  lds_get_fe<FE_LIMBS>(S.part[k][2], p.z.v, l);
  inf = S.pinf[k][l] != 0;
  return p;
}

// Table {1..NT} * P (P affine in its own coordinates: the formulas never use the curve's b)
// on one global Z (co-Z additions, backward rescale; core.cuh ecmult_core). Returns zeta.
// A wave of this kernel usually has its SIMD to itself, so nothing hides a dependent load's
// latency: the backward pass loads entry i - 1 while it rescales entry i.
template <int NT>
DEV fe build_table_mid(uint32_t* tab, uint32_t* zr, const ge& P, uint32_t l) {
  store_pt(tab + (size_t)l * PT_WORDS, P);
  gej D;
  ge B;
  gej_dblu(D, B, P);
  store_fe(zr + (size_t)l * ZR_WORDS, D.z);  // Z_2 / Z_1 = 2y
  ge T;
  T.x = D.x;
  T.y = D.y;
  store_pt(tab + (size_t)(1 * MID_L + l) * PT_WORDS, T);
#pragma unroll 1
  for (int i = 2; i < NT; ++i) {
    const fe r = gej_zaddu(T, B);  // T = (i+1) P
    store_pt(tab + (size_t)(i * MID_L + l) * PT_WORDS, T);
    store_fe(zr + (size_t)((i - 1) * MID_L + l) * ZR_WORDS, r);
  }
  fe rho = fe_one();
  ge Jn = load_pt(tab + (size_t)((NT - 2) * MID_L + l) * PT_WORDS);
  fe rn = load_fe(zr + (size_t)((NT - 2) * MID_L + l) * ZR_WORDS);
#pragma unroll 1
  for (int i = NT - 2; i >= 0; --i) {
    const ge J = Jn;
    const fe r = rn;  // Z_{i+2} / Z_{i+1}
    if (i > 0) {
      Jn = load_pt(tab + (size_t)((i - 1) * MID_L + l) * PT_WORDS);
      rn = load_fe(zr + (size_t)((i - 1) * MID_L + l) * ZR_WORDS);
    }
    rho = i == NT - 2 ? r : fe_mul(rho, r);  // Z_NT / Z_{i+1}
    const fe r2 = fe_sqr(rho);
    ge a;
    a.x = fe_mul(J.x, r2);
    a.y = fe_mul(J.y, fe_mul(r2, rho));
    store_pt(tab + (size_t)(i * MID_L + l) * PT_WORDS, a);
  }
  return rho;  // Z_NT / Z_1 with Z_1 = 1
}

// Windows [0, NW) of the GLV halves selected by JM (bit 0: R digits d0, bit 1: lambda R digits
// d1, lambda (x, y) = (beta x, y)), Horner from the top window, BITS doublings per window. The
// next window's table entries are loaded before this window's additions, so their latency hides
// behind the additions and the next BITS doublings.
template <bool CHECKED, int BITS, int NT, int NW, int JM>
DEV void strauss_mid(gej& acc, bool& inf, const uint32_t* tab, const int8_t (*d0)[MID_L], const int8_t (*d1)[MID_L],
                     uint32_t l, const Diag& dg) {
  inf = true;
  acc.x = fe_zero();
  acc.y = fe_zero();
  acc.z = fe_zero();
  auto entry = [&](int d) {
    const int a = d < 0 ? -d : d;
    return load_pt(tab + (size_t)((a > 0 ? a - 1 : 0) * MID_L + l) * PT_WORDS);
  };
  int dn0 = (JM & 1) ? (int)d0[NW - 1][l] : 0, dn1 = (JM & 2) ? (int)d1[NW - 1][l] : 0;
  ge pn0, pn1;
  if (JM & 1) pn0 = entry(dn0);
  if (JM & 2) pn1 = entry(dn1);
#pragma unroll 1
  for (int w = NW - 1; w >= 0; --w) {
    if (w != NW - 1) {
#pragma unroll 1
      for (int k = 0; k < BITS; ++k) acc = gej_double(acc);
    }
    const int c0 = dn0, c1 = dn1;
    ge p0 = pn0, p1 = pn1;
    if (w > 0) {
      if (JM & 1) {
        dn0 = (int)d0[w - 1][l];
        pn0 = entry(dn0);
      }
      if (JM & 2) {
        dn1 = (int)d1[w - 1][l];
        pn1 = entry(dn1);
      }
    }
    if (JM & 1) {
      if (CHECKED) add_step(acc, inf, neg_if(p0, c0 < 0), c0 != 0, dg, EGES_DIAG_MID_EXC);
      else add_step_fast(acc, inf, neg_if(p0, c0 < 0), c0 != 0);
    }
    if (JM & 2) {
      p1.x = fe_mul(p1.x, fe_const(FE_BETA));
      if (CHECKED) add_step(acc, inf, neg_if(p1, c1 < 0), c1 != 0, dg, EGES_DIAG_MID_EXC);
      else add_step_fast(acc, inf, neg_if(p1, c1 < 0), c1 != 0);
    }
  }
}
template <int BITS, int NT, int NW, int JM>
DEV void strauss_mid_exact(gej& acc, bool& inf, const uint32_t* tab, const int8_t (*d0)[MID_L],
                           const int8_t (*d1)[MID_L], uint32_t l, const Diag& dg) {
  strauss_mid<false, BITS, NT, NW, JM>(acc, inf, tab, d0, d1, l, dg);
  if (dg.force || __any(!inf && fe_is_zero(acc.z))) {
    diag_bump(dg, EGES_DIAG_MID_REDO);
    strauss_mid<true, BITS, NT, NW, JM>(acc, inf, tab, d0, d1, l, dg);
  }
}

// u G by the comb table (k_recover_lat.hip strauss_gcomb, lane-serial): one mixed addition per
// nonzero 16-bit digit, no doublings, true curve; the next digit's entry is loaded ahead.
template <bool CHECKED>
DEV void comb_mid(gej& acc, bool& inf, const sc& u, const uint32_t* gcomb, const Diag& dg) {
  inf = true;
  acc.x = fe_zero();
  acc.y = fe_zero();
  acc.z = fe_zero();
  auto digit = [&](int k) { return (int)((u.v[k >> 1] >> (16 * (k & 1))) & 0xFFFFu); };
  auto entry = [&](int k, int d) { return load_pt(gcomb + ((size_t)k * CTAB + (d > 0 ? d - 1 : 0)) * PT_WORDS); };
  int dn = digit(0);
  ge pn = entry(0, dn);
#pragma unroll 1
  for (int k = 0; k < CWIN; ++k) {
    const int d = dn;
    const ge p = pn;
    if (k + 1 < CWIN) {
      dn = digit(k + 1);
      pn = entry(k + 1, dn);
    }
    if (CHECKED) add_step(acc, inf, p, d != 0, dg, EGES_DIAG_MID_EXC);
    else add_step_fast(acc, inf, p, d != 0);
  }
}

// Exact general addition a + b (add-2007-bl, Z3 = 2 Z1 Z2 H), infinity flags in and out; a == b
// doubles, a == -b gives infinity (group_impl.h:414-461's cases). In: X m1, Y <= 2, Z <= 2.
// Out: X, Y m1, Z m2.
DEV gej join_mid(const gej& a, bool ainf, const gej& b, bool binf, bool& rinf, const Diag& dg) {
  const fe Z1Z1 = fe_sqr(a.z), Z2Z2 = fe_sqr(b.z);
  const fe U1 = fe_mul(a.x, Z2Z2), U2 = fe_mul(b.x, Z1Z1);
  const fe S1 = fe_mul(fe_mul(a.y, b.z), Z2Z2), S2 = fe_mul(fe_mul(b.y, a.z), Z1Z1);
  const fe H = fe_normalize_weak(fe_sub<1>(U2, U1));
  const fe Rd = fe_normalize_weak(fe_sub<1>(S2, S1));
  const fe H2 = fe_add(H, H), R2 = fe_add(Rd, Rd);
  const fe I = fe_sqr(H2);           // (2H)^2
  const fe J = fe_mul(H, I);
  const fe V = fe_mul(U1, I);
  gej r;
  r.x = fe_sqr_sub<2>(R2, fe_add(J, fe_add(V, V)));               // r^2 - J - 2V
  r.y = fe_mul_sub<1, 1>(R2, fe_sub<1>(V, r.x), fe_mul(S1, J));   // r (V - X3) - 2 S1 J
  const fe zh = fe_mul(fe_mul(a.z, b.z), H);
  r.z = fe_add(zh, zh);
  const bool exc = !ainf && !binf && fe_is_zero(H);
  const bool rz = fe_is_zero(Rd);
  if (__any(exc)) {
    diag_bump(dg, EGES_DIAG_MID_JOIN);
    r = gej_select(exc && rz, gej_double(a), r);
  }
  rinf = ainf ? binf : (binf ? false : (exc && !rz));
  return gej_select(ainf, b, gej_select(binf, a, r));
}

// signed fixed-window recoding of a GLV half (core.cuh recode) into this lane's column:
// SPLIT windows of 5 bits into lo, then (carry included) 4-bit windows into hi
DEV void recode_mid(const glv_half& h, int8_t (*lo)[MID_L], int8_t (*hi)[MID_L], uint32_t l) {
  uint32_t m[5];
#pragma unroll
  for (int i = 0; i < 5; ++i) m[i] = h.mag[i];
  int carry = 0;
#pragma unroll 1
  for (int w = 0; w < MID_W0 + MID_HWIN; ++w) {
    const int W = w < MID_W0 ? RBITS : MID_HBITS;
    const uint32_t mask = (1u << W) - 1;
    int v = (int)(m[0] & mask) + carry;
    carry = v > (1 << (W - 1)) ? 1 : 0;
    v -= carry << W;
    const int8_t d = (int8_t)(h.neg ? -v : v);
    if (w < MID_W0) lo[w][l] = d;
    else hi[w - MID_W0][l] = d;
#pragma unroll
    for (int i = 0; i < 4; ++i) m[i] = (m[i] >> W) | (m[i + 1] << (32 - W));
    m[4] >>= W;
  }
}

template <class ST>
DEV void recover_mid_body(const RecoverParams& prm, uint64_t* stamps) {
  gate_wait(prm);
  __shared__ MidLds S;
  ST st_;
  const Diag dg = diag_of(prm);
  const uint32_t l = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint32_t idx = blockIdx.x * MID_L + l;
  const bool live = idx < prm.n;
  if (threadIdx.x < MF_N) S.flag[threadIdx.x] = 0u;
  __syncthreads();  // the only barrier
  const uint32_t pidx = live ? idx : prm.n - 1;
  const LatParse q = prm.snd_r ? sender_parse_lane(prm, pidx) : lat_parse(prm, pidx);
  // diagnostic build: per-wave phase ticks, row blockIdx * 4 + wave (tools/phases_mid.py)
  auto stamp_out = [&] {
    if constexpr (!std::is_same<ST, NoStamp>::value) {
      if (l == 0) {
#pragma unroll
        for (int i = 0; i < 8; ++i) stamps[((size_t)blockIdx.x * 4 + wv) * 8 + i] = st_.acc[i];
      }
    }
  };
  const bool pok = live && q.ok;
  // signatures that fail the parse carry the generator's x (even y): every step stays defined
  const ge G = gen_point();
  const fe x = fe_select(pok, fe_from_u256(q.xr), G.x);
  const fe c = fe_normalize_weak(fe_add(fe_mul(fe_sqr(x), x), fe_from_u32(7)));  // x^3 + 7
  uint32_t* ws = prm.ws + (size_t)blockIdx.x * MID_WS_WORDS;
  if (wv == 1) {  // ---- S: scalars, digits, y, u1 G
    st_.mark(0);
    const sc R = sc_select(pok, q.R, sc_one());
    const sc rinv = sc_inv(R);
    const sc u1 = sc_neg(sc_mul(rinv, q.Z));  // main_impl.h:114-117
    const sc u2 = sc_select(pok, sc_mul(rinv, q.Sv), sc_one());
    st_.mark(1);
    glv_half h1, h2;
    glv_split(h1, h2, u2);
    recode_mid(h1, S.lo[0], S.hi[0], l);
    recode_mid(h2, S.lo[1], S.hi[1], l);
    MFLAG_SET(MF_DIG);
    st_.mark(2);
    ge Rp;
    const bool yok = ge_set_xo(Rp, x, pok && (q.recid & 1u) != 0);  // ge_set_xo_var, group_impl.h:216-237
    lds_put_fe<FE_LIMBS>(S.y, Rp.y.v, l);
    S.yok[l] = yok ? 1u : 0u;
    MFLAG_SET(MF_Y);
    st_.mark(3);
    const uint32_t* gcomb = prm.gtab + (size_t)2 * GTAB * PT_WORDS;
    gej Ga;
    bool ginf;
    comb_mid<false>(Ga, ginf, u1, gcomb, dg);
    if (dg.force || __any(!ginf && fe_is_zero(Ga.z))) {
      diag_bump(dg, EGES_DIAG_MID_REDO);
      comb_mid<true>(Ga, ginf, u1, gcomb, dg);
    }
    put_part_ls(S, 0, Ga, ginf, l);
    MFLAG_SET(MF_G);
    st_.mark(4);
    stamp_out();
    return;
  }
  // R' = (c x, c^2): R's image on E' (no square root on this path)
  ge Rp;
  Rp.x = fe_mul(c, x);
  Rp.y = fe_sqr(c);
  if (wv >= 2) {  // ---- B / C: D = 2^(5 MID_W0) R', its table, the high windows of one half
    const int j = (int)wv - 2;
    st_.mark(0);
    gej D;
    D.x = Rp.x;
    D.y = Rp.y;
    D.z = fe_one();
#pragma unroll 1
    for (int k = 0; k < RBITS * MID_W0; ++k) D = gej_double(D);  // R' has odd order: never exceptional
    st_.mark(1);
    ge Dp;
    Dp.x = D.x;
    Dp.y = D.y;
    uint32_t* tab = ws + (j ? MID_TAB_C : MID_TAB_B);
    const fe zd = build_table_mid<MID_HTAB>(tab, ws + (j ? MID_ZR_C : MID_ZR_B), Dp, l);
    const fe scale = fe_mul(zd, D.z);
    st_.mark(2);
    MFLAG_WAIT(MF_DIG);
    st_.mark(3);
    gej H;
    bool hinf;
    if (j == 0) strauss_mid_exact<MID_HBITS, MID_HTAB, MID_HWIN, 1>(H, hinf, tab, S.hi[0], S.hi[1], l, dg);
    else strauss_mid_exact<MID_HBITS, MID_HTAB, MID_HWIN, 2>(H, hinf, tab, S.hi[0], S.hi[1], l, dg);
    H.z = fe_mul(H.z, scale);  // E' coordinates
    put_part_ls(S, 1 + j, H, hinf, l);
    MFLAG_SET(j ? MF_HC : MF_HB);
    st_.mark(4);
    stamp_out();
    return;
  }
  // ---- A: the R' table, the low windows of both halves, then the joins and the address
  uint32_t* tab = ws + MID_TAB_A;
  st_.mark(0);
  const fe zeta = build_table_mid<PTAB>(tab, ws + MID_ZR_A, Rp, l);
  st_.mark(3);
  MFLAG_WAIT(MF_DIG);
  st_.mark(1);
  gej A;
  bool ainf;
  strauss_mid_exact<RBITS, PTAB, MID_W0, 3>(A, ainf, tab, S.lo[0], S.lo[1], l, dg);
  st_.mark(4);
  // back to E: an E' Jacobian point (X, Y, Z) is (X, Y, Z y) on E; the table curve adds zeta.
  // A + u1 G first (both are usually ready before the high waves finish), then the high parts.
  MFLAG_WAIT(MF_Y);
  fe y;
  lds_get_fe<FE_LIMBS>(S.y, y.v, l);
  const bool yok = S.yok[l] != 0;
  A.z = fe_mul(A.z, fe_mul(zeta, y));
  bool binf, cinf, ginf, hinf, qinf;
  MFLAG_WAIT(MF_G);
  st_.mark(7);
  const gej Gp = get_part_ls(S, 0, ginf, l);
  gej Q = join_mid(A, ainf, Gp, ginf, qinf, dg);
  st_.mark(2);
  MFLAG_WAIT(MF_HB);
  MFLAG_WAIT(MF_HC);
  st_.mark(7);
  gej Hb = get_part_ls(S, 1, binf, l), Hc = get_part_ls(S, 2, cinf, l);
  Hb.z = fe_mul(Hb.z, y);
  Hc.z = fe_mul(Hc.z, y);
  const gej H = join_mid(Hb, binf, Hc, cinf, hinf, dg);
  Q = join_mid(Q, qinf, H, hinf, qinf, dg);
  st_.mark(2);
  const bool fault = ho_failed(&S.flag[MF_ERR], dg);  // after A's last wait
  const bool ok = pok && yok && !qinf && !fault;  // main_impl.h:120
  // affine, serialize, address
  // (a zero factor would zero the whole wave's batch inversion: such a lane, which the exceptional-sum
  // argument excludes, takes 1 and keeps its own wrong value to itself)
  const fe zq = fe_select(ok && !fe_is_zero(Q.z), Q.z, fe_one());
  const fe zi = fe_inv_wave(zq);
  const fe zi2 = fe_sqr(zi);
  uint32_t X[8], Y[8];
  fe_to_u256(X, fe_normalize(fe_mul(Q.x, zi2)));
  fe_to_u256(Y, fe_normalize(fe_mul(Q.y, fe_mul(zi2, zi))));
  st_.mark(5);
  if (live) {
    const uint32_t pre_st = (q.meta >> 8) & 0xffu;
    prm.status[idx] = (uint8_t)(fault ? ST_ENGINE_FAULT : pre_st != ST_OK ? pre_st : (ok ? ST_OK : ST_RECOVER_FAILED));
    if (prm.addr) {
      uint32_t a[5];
      pub_address(a, X, Y);
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
  }
  st_.mark(6);
  stamp_out();
}

// ================================================================== bucket form
// The same 64 signatures per 4-wave workgroup, with u2 R computed bottom-up so the doubling
// chain carries no additions and needs no table:
//
//   wave 0 "X"   P_0 = R' (affine on E'), P_{3k} = 2^(3k) R' by 126 doublings; publishes
//                every third point into an LDS ring (BK_RING slots, flow-controlled by the
//                consumers' counters)
//   wave 2 "Y1"  for every published P_{3k}: bucket[|d1_k|] += sign(d1_k) P_{3k}, d1 the signed
//                3-bit digits of the R half; then Q1 = sum_v v bucket[v] (running sums, exact
//                joins), Q = Q1 + Q2 (E'), Q *= y (E), Q += u1 G, Z^-1, affine, address, stores
//   wave 3 "Y2"  the same for the lambda R half: buckets of d2_k P_{3k}, then Q2 = lambda (sum)
//                by (X, Y, Z) -> (beta X, Y, Z) once, and hands Q2 to Y1
//   wave 1 "S"   r^-1, u1, u2, GLV split, the digits; R's y; u1 G by the comb
//
// The critical path is X's 126 doublings plus Y1's tail (bucket sums, two joins, Z^-1, Keccak);
// the windowed form's chain (D = 2^75 R', its table, 14 windows with their additions, then the
// same tail) was ~20 % longer.
//
// Exceptional sums. A bucket of half h collects +-2^(3j) R'_h over distinct j in increasing
// order: before window k its value is m R'_h with 0 < |m| <= sum_{j<k} 2^(3j) < 2^(3k), so
// m == +-2^(3k) (mod n) is impossible (|m|, 2^(3k) < n / 2) and the unchecked general
// additions never meet a == +-b (tests/ecmodel.py `bucket`, tests/test_exceptional_model.py).
// The bucket sum Q_h = (B1 + B3) + 2 ((B2 + B3) + 2 B4) cannot meet them either: every join
// adds signed-binary integers whose +-1 digits sit at distinct bit positions (3j, 3j + 1,
// 3j + 2 for the windows j of each bucket), so a == +-b only when both are empty. Q_1 + Q_2
// would need k1 == lambda k2 for the split's own output (never, test_exceptional_model.py);
// the final join with u1 G is reachable (u1 chosen against u2 R). All joins are exact
// additions (join_mid) anyway. A lane that ends with Z == 0 although it is valid would
// contradict the argument: it is counted (EGES_DIAG_MID_EXC; the tests require 0).
constexpr int BK_BITS = 3;
// |k1|, |k2| < 0.64 * 2^128 for the Babai-rounded split (sc.cuh glv_split; the bound is
// (|a1| + |a2|) / 2 and (|b1| + a1) / 2 over the lattice basis, tests/test_exceptional_model.py):
// 128 bits + the recoding carry, 43 windows, 126 doublings
constexpr int BK_WIN = (129 + BK_BITS - 1) / BK_BITS;
constexpr int BK_NB = 1 << (BK_BITS - 1);             // buckets for |digit| = 1..4
constexpr int BK_RING = 10;
constexpr int GJ_WORDS = 3 * FE_LIMBS;

enum {
  BF_DIG = 0, BF_Y, BF_G, BF_Q2, BF_PUB, BF_CON0, BF_CON1, BF_PARSED, BF_STAGE_FREE, BF_FIN0, BF_FIN1, BF_A0, BF_A1,
  BF_ERR, BF_N
};
// ring slots that hold wave X's partial bucket sums B1 + B3 of each half once the ring is drained
// (their points, 33 and 34, are consumed by both halves before either finishes)
constexpr int BK_ASLOT = 3;
static_assert(BK_RING > BK_ASLOT + 1 && BK_WIN - BK_RING > BK_ASLOT + 1, "partial-sum slots");

constexpr int BK_STAGE_WORDS = 2 * GJ_WORDS * MID_L;  // wire form: staged encodings (13.5 KB)
// Two-per-CU variant (G2, round 6, VERDICT r5 item 3: the 16k-32k band): the ring and the two
// parts live in a per-workgroup area of the device workspace instead of LDS (BK2_WS_WORDS, the
// same [word][lane] layout, so every access stays coalesced): ~76 KB of LDS per workgroup and
// 215 registers, two workgroups per CU, one generation up to 128 x CUs signatures. No wire form.
constexpr size_t BK2_RING_WORDS = (size_t)BK_RING * GJ_WORDS * MID_L;
constexpr size_t BK2_WS_WORDS = BK2_RING_WORDS + (size_t)2 * GJ_WORDS * MID_L;
template <bool G2>
struct BktLdsT {
  uint32_t ring[G2 ? 1 : BK_RING][GJ_WORDS][MID_L];  // published P_{3k}, slot k % BK_RING (G2: unused)
  uint32_t bucket[2][BK_NB][GJ_WORDS][MID_L];        // per half; lanes index their own bucket
  union {
    uint32_t part[G2 ? 1 : 2][GJ_WORDS][MID_L];      // 0: u1 G (E), 1: Q2 (E') (G2: unused)
    uint32_t stage[G2 ? 1 : BK_STAGE_WORDS];         // wire form: the workgroup's encodings, until
  } u;                                               //   wave S has hashed them (BF_STAGE_FREE)
  uint32_t meta[MID_L];                              // wire form: wave S's pre-check meta and ok
  uint8_t pok[MID_L];
  uint32_t y[FE_LIMBS][MID_L];
  uint8_t binf[2][BK_NB][MID_L];
  uint8_t pinf[2][MID_L];
  uint8_t ainf[2][MID_L];
  uint8_t yok[MID_L];
  int8_t dig[2][BK_WIN][MID_L];
  uint32_t flag[BF_N];
};
using BktLds = BktLdsT<false>;
static_assert(sizeof(BktLds) <= 160 * 1024, "bucket form LDS");
static_assert(2 * sizeof(BktLdsT<true>) <= 160 * 1024, "bucket form, two per CU");


DEV void lds_put_gej(uint32_t (*a)[MID_L], const gej& p, uint32_t l) {
  lds_put_fe<FE_LIMBS>(a, p.x.v, l);
  lds_put_fe<FE_LIMBS>(a + FE_LIMBS, p.y.v, l);
  lds_put_fe<FE_LIMBS>(a + 2 * FE_LIMBS, p.z.v, l);
}
DEV gej lds_get_gej(const uint32_t (*a)[MID_L], uint32_t l) {
  gej p;
  lds_get_fe<FE_LIMBS>(a, p.x.v, l);
  lds_get_fe<FE_LIMBS>(a + FE_LIMBS, p.y.v, l);
  lds_get_fe<FE_LIMBS>(a + 2 * FE_LIMBS, p.z.v, l);
  return p;
}

// the ring slots and parts: LDS, or (G2) the workgroup's area of the device workspace
template <bool G2>
struct BktStore {
  BktLdsT<G2>& S;
  uint32_t* g;  // G2: ring [BK_RING][GJ_WORDS][MID_L], then part [2][GJ_WORDS][MID_L]
  DEV void ring_put(uint32_t slot, const gej& p, uint32_t l) {
    if constexpr (G2) gput(g + (size_t)slot * GJ_WORDS * MID_L, p, l);
    else lds_put_gej(S.ring[slot], p, l);
  }
  DEV gej ring_get(uint32_t slot, uint32_t l) {
    if constexpr (G2) return gget(g + (size_t)slot * GJ_WORDS * MID_L, l);
    else return lds_get_gej(S.ring[slot], l);
  }
  DEV void part_put(int i, const gej& p, uint32_t l) {
    if constexpr (G2) gput(g + BK2_RING_WORDS + (size_t)i * GJ_WORDS * MID_L, p, l);
    else lds_put_gej(S.u.part[i], p, l);
  }
  DEV gej part_get(int i, uint32_t l) {
    if constexpr (G2) return gget(g + BK2_RING_WORDS + (size_t)i * GJ_WORDS * MID_L, l);
    else return lds_get_gej(S.u.part[i], l);
  }
  // [GJ_WORDS][MID_L] in global memory: word w of lane l at a[w * MID_L + l] (coalesced)
  static DEV void gput(uint32_t* a, const gej& p, uint32_t l) {
#pragma unroll
    for (int i = 0; i < FE_LIMBS; ++i) {
      a[i * MID_L + l] = p.x.v[i];
      a[(FE_LIMBS + i) * MID_L + l] = p.y.v[i];
      a[(2 * FE_LIMBS + i) * MID_L + l] = p.z.v[i];
    }
  }
  static DEV gej gget(const uint32_t* a, uint32_t l) {
    gej p;
#pragma unroll
    for (int i = 0; i < FE_LIMBS; ++i) {
      p.x.v[i] = a[i * MID_L + l];
      p.y.v[i] = a[(FE_LIMBS + i) * MID_L + l];
      p.z.v[i] = a[(2 * FE_LIMBS + i) * MID_L + l];
    }
    return p;
  }
};

// Flags and LDS counters (handoff.cuh): the producer publishes a flag or a running count after
// a workgroup release fence, consumers wait (bounded) until it reaches k and acquire.
#define BFLAG_SET(k) ho_set(&S.flag[k], 1u, ho_skip(prm, k))
#define BFLAG_WAIT(k) ho_wait<2>(&S.flag[k], 1u, &S.flag[BF_ERR])
#define CNT_SET(k, v) ho_set(&S.flag[k], (v))
#define CNT_WAIT(k, v) ho_wait<1>(&S.flag[k], (v), &S.flag[BF_ERR])

// a + b, both Jacobian, neither at infinity, a != +-b (add-2007-bl, join_mid without the checks).
// In: X m1, Y <= 2, Z <= 2. Out: X, Y m1, Z m2.
DEV gej gej_add_fast(const gej& a, const gej& b) {
  const fe Z1Z1 = fe_sqr(a.z), Z2Z2 = fe_sqr(b.z);
  const fe U1 = fe_mul(a.x, Z2Z2);
  const fe S1 = fe_mul(fe_mul(a.y, b.z), Z2Z2);
  const fe H = fe_mul_sub<1>(b.x, Z1Z1, U1);                   // U2 - U1
  const fe Rd = fe_mul_sub<1>(fe_mul(b.y, a.z), Z1Z1, S1);     // S2 - S1
  const fe H2 = fe_add(H, H), R2 = fe_add(Rd, Rd);
  const fe I = fe_sqr(H2);
  const fe J = fe_mul(H, I);
  const fe V = fe_mul(U1, I);
  gej r;
  r.x = fe_sqr_sub<2>(R2, fe_add(J, fe_add(V, V)));
  r.y = fe_mul_sub<1, 1>(R2, fe_sub<1>(V, r.x), fe_mul(S1, J));
  const fe zh = fe_mul(fe_mul(a.z, b.z), H);
  r.z = fe_add(zh, zh);
  return r;
}

// signed BK_BITS-bit windows of a GLV half into this lane's column (core.cuh recode)
DEV void recode_bk(const glv_half& h, int8_t (*out)[MID_L], uint32_t l) {
  uint32_t m[5];
#pragma unroll
  for (int i = 0; i < 5; ++i) m[i] = h.mag[i];
  int carry = 0;
#pragma unroll 1
  for (int w = 0; w < BK_WIN; ++w) {
    constexpr uint32_t mask = (1u << BK_BITS) - 1;
    int v = (int)(m[0] & mask) + carry;
    carry = v > (1 << (BK_BITS - 1)) ? 1 : 0;
    v -= carry << BK_BITS;
    out[w][l] = (int8_t)(h.neg ? -v : v);
#pragma unroll
    for (int i = 0; i < 4; ++i) m[i] = (m[i] >> BK_BITS) | (m[i + 1] << (32 - BK_BITS));
    m[4] >>= BK_BITS;
  }
}

// Wire form: the workgroup's encodings [lo, hi) (relative to wire_raw, which is 4-byte aligned)
// copied into S.u.stage by all 256 threads with coalesced dword loads (from pinned host memory
// these are long PCIe reads instead of one dependent byte load per RLP header); bytes past the
// stage's capacity stay in global memory. Returns the staged window [a0, end).
DEV void wire_stage(BktLds& S, const RecoverParams& prm, uint64_t& a0, uint64_t& end) {
  const uint32_t i0 = blockIdx.x * MID_L;
  const uint32_t cnt = prm.n - i0 < (uint32_t)MID_L ? prm.n - i0 : (uint32_t)MID_L;
  const uint64_t* off = prm.wire_off + prm.wire_first;
  const uint64_t base = prm.wire_off[0], lo = off[i0] - base, hi = off[i0 + cnt] - base;
  a0 = lo & ~(uint64_t)3;
  end = a0;
  if (hi <= lo || off[i0] < base) return;  // malformed offsets: every item reads global memory
  const uint64_t full = (hi - a0) / 4;  // whole dwords inside [a0, hi): no read past the batch
  const uint32_t nw = full < (uint64_t)BK_STAGE_WORDS ? (uint32_t)full : (uint32_t)BK_STAGE_WORDS;
  const uint32_t* src = reinterpret_cast<const uint32_t*>(prm.wire_raw + a0);
#pragma unroll 4
  for (uint32_t w = threadIdx.x; w < nw; w += MID_WG) S.u.stage[w] = src[w];
  end = a0 + 4 * (uint64_t)nw;
  if (nw == full && nw < (uint32_t)BK_STAGE_WORDS) {  // the tail bytes of the last dword
    const uint32_t tb = (uint32_t)(hi - end);
    if (threadIdx.x < tb) reinterpret_cast<uint8_t*>(S.u.stage)[4 * nw + threadIdx.x] = prm.wire_raw[end + threadIdx.x];
    end = hi;
  }
}

// Wire form, wave S, one lane per transaction: tx_rows_kernel's decode (k_txhash.hip, rlp.cuh)
// and prep_sender_kernel's classification (sender.cuh) of item idx. Fills q as lat_parse would
// (except q.Z: the signing hash comes later, from m).
// (Not inlined: the decoder's ten item heads would otherwise raise the register pressure of the
// whole kernel, the doubling and bucket loops included.)
__device__ __attribute__((noinline)) void wire_parse(const BktLds& S, const RecoverParams& prm, uint32_t idx,
                                                     uint64_t a0, uint64_t end, LatParse& q, Payload& m) {
  const uint64_t base = prm.wire_off[0], a = prm.wire_off[prm.wire_first + idx], e = prm.wire_off[prm.wire_first + idx + 1];
  const bool span_ok = e >= a && a >= base;
  const uint64_t ra = span_ok ? a - base : 0, len = span_ok ? e - a : 0;
  const uint8_t* p = (ra >= a0 && ra + len <= end) ? reinterpret_cast<const uint8_t*>(S.u.stage) + (ra - a0)
                                                   : prm.wire_raw + ra;
  wire_item(p, len, span_ok, prm.wire_signer, prm.wire_chain_id, q, m);
}

__device__ __attribute__((noinline)) void wire_sighash(const Payload& m, uint8_t* h) { keccak256_payload(m, h); }

// Wire form, wave X: only R's 32 bytes (item 8 of the txdata list) as x, by walking the item
// heads. An item S rejects (decode, V / chain id, range checks) is invalid whatever x is (its
// result is discarded), and for every valid one this is S's r: the chain needs no S flag.
__device__ __attribute__((noinline)) bool wire_r_only(const BktLds& S, const RecoverParams& prm, uint32_t idx,
                                                      uint64_t a0, uint64_t end, uint32_t xr[8]) {
  const uint64_t base = prm.wire_off[0], a = prm.wire_off[prm.wire_first + idx], e = prm.wire_off[prm.wire_first + idx + 1];
  if (!(e >= a && a >= base)) return false;
  const uint64_t ra = a - base, len = e - a;
  const uint8_t* p = (ra >= a0 && ra + len <= end) ? reinterpret_cast<const uint8_t*>(S.u.stage) + (ra - a0)
                                                   : prm.wire_raw + ra;
  RlpHead L{}, f{};
  bool ok = rlp_head(p, 0, len, L) && L.kind == RK_LIST;
  uint64_t pos = L.off;
  const uint64_t lend = L.off + L.size;
#pragma unroll 1
  for (int k = 0; k < 9 && ok; ++k) {
    ok = rlp_head(p, pos, lend, f);
    pos = f.next;
  }
  uint8_t b[32];
  ok = ok && rlp_to_be32(p, f, b);
  if (ok) limbs_from_be32(xr, b);
  return ok;
}

// VerifySignature mode (VERIFY): item idx's signature, message and public key as the lane-serial
// verify kernel parses them (k_verify.hip verify_parse; eckey_impl.h:17-34, secp256k1.c:293-308):
// q.R = r, q.Sv = s, q.Z = z, q.xr = the key's x, q.ok = the signature and key checks that need
// no field arithmetic; py / c65 / odd for wave S's y (given, or the root of a 33-byte key).
DEV void verify_parse_lane(const RecoverParams& prm, uint32_t idx, LatParse& q, uint32_t py[8], bool& c65, bool& odd) {
  uint32_t l[8];
  bool ovr, ovs, ovz;
  limbs_from_be32(l, prm.v_sig + (size_t)idx * 64);
  q.R = sc_from_limbs(l, ovr);
  limbs_from_be32(l, prm.v_sig + (size_t)idx * 64 + 32);
  q.Sv = sc_from_limbs(l, ovs);
  limbs_from_be32(l, prm.v_msg + (size_t)idx * 32);
  q.Z = sc_from_limbs(l, ovz);  // the message reduced mod n
  const bool sig_ok = !ovr && !ovs && !sc_is_high(q.Sv) && !sc_is_zero(q.R) && !sc_is_zero(q.Sv);
  const uint32_t plen = prm.v_publen[idx];
  const uint8_t* pk = prm.v_pub + (size_t)idx * 65;
  const uint32_t pfx = pk[0];
  limbs_from_be32(q.xr, pk + 1);
  if (plen == 65) {
    limbs_from_be32(py, pk + 33);
  } else {
#pragma unroll
    for (int k = 0; k < 8; ++k) py[k] = 0;
  }
  const bool x_ok = !u256_ge(q.xr, FE_P), y_ok = !u256_ge(py, FE_P);
  const bool c33 = plen == 33 && (pfx == 2 || pfx == 3);
  c65 = plen == 65 && (pfx == 4 || pfx == 6 || pfx == 7);
  const bool hybrid_bad = (pfx == 6 || pfx == 7) && ((py[0] & 1u) != (pfx == 7 ? 1u : 0u));
  q.ok = sig_ok && ((c33 && x_ok) || (c65 && x_ok && y_ok && !hybrid_bad));
  odd = pfx == 3;
  q.meta = 0;
  q.recid = 0;
}

template <class ST, bool VERIFY = false, bool G2 = false>
DEV void recover_bkt_body(const RecoverParams& prm, uint64_t* stamps) {
  gate_wait(prm);
  __shared__ BktLdsT<G2> S;
  BktStore<G2> rg{S, G2 ? prm.ws + (size_t)blockIdx.x * BK2_WS_WORDS : nullptr};
  ST st_;
  const Diag dg = diag_of(prm);
  const uint32_t l = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint32_t idx = blockIdx.x * MID_L + l;
  const bool live = idx < prm.n;
  const bool wire = !VERIFY && !G2 && prm.wire_raw != nullptr;  // kernel-uniform
  uint64_t stage_a0 = 0, stage_end = 0;
  if (threadIdx.x < BF_N) S.flag[threadIdx.x] = 0u;
  if constexpr (!G2)
    if (wire) wire_stage(S, prm, stage_a0, stage_end);
  __syncthreads();  // the only barrier
  LatParse q;
  Payload m;
  uint32_t vpy[8];
  bool vc65 = false, vodd = false;
  if (VERIFY) {
    verify_parse_lane(prm, live ? idx : prm.n - 1, q, vpy, vc65, vodd);
  } else if (!wire) {
    q = prm.snd_r ? sender_parse_lane(prm, live ? idx : prm.n - 1) : lat_parse(prm, live ? idx : prm.n - 1);
  } else if (wv == 1) {
    if constexpr (!G2) wire_parse(S, prm, live ? idx : prm.n - 1, stage_a0, stage_end, q, m);
    S.meta[l] = q.meta;
    S.pok[l] = live && q.ok ? 1u : 0u;
    BFLAG_SET(BF_PARSED);
  } else if (wv == 0) {  // R's x straight from the encoding, without waiting for S's checks
#pragma unroll 1
    for (uint32_t k = 0; k < prm.test_delay_x; ++k) __builtin_amdgcn_s_sleep(127);  // tests only
    if constexpr (!G2) q.ok = live && wire_r_only(S, prm, idx, stage_a0, stage_end, q.xr);
  } else {
    q.ok = false;  // Y waves: read from LDS at the end
  }
  auto stamp_out = [&] {
    if constexpr (!std::is_same<ST, NoStamp>::value) {
      if (l == 0) {
#pragma unroll
        for (int i = 0; i < 8; ++i) stamps[((size_t)blockIdx.x * 4 + wv) * 8 + i] = st_.acc[i];
      }
    }
  };
  const bool pok = live && q.ok;
  const ge G = gen_point();
  const fe x = fe_select(pok, fe_from_u256(q.xr), G.x);
  if (wv == 1) {  // ---- S: scalars, digits, y, u1 G
    st_.mark(0);
    // recovery: r^-1, u2 = s / r, u1 = -z / r (main_impl.h:114-117); verification: s^-1,
    // u2 = r / s, u1 = z / s (ecdsa_impl.h:203-271)
    const sc R = sc_select(pok, VERIFY ? q.Sv : q.R, sc_one());
    const sc rinv = sc_inv(R);
    const sc u2 = sc_select(pok, sc_mul(rinv, VERIFY ? q.R : q.Sv), sc_one());
    st_.mark(1);
    glv_half h1, h2;
    glv_split(h1, h2, u2);
    recode_bk(h1, S.dig[0], l);
    recode_bk(h2, S.dig[1], l);
    BFLAG_SET(BF_DIG);
    st_.mark(2);
    if (wire) {  // the signing hash (FrontierSigner / EIP155Signer.Hash) of the encoding, then z
      uint8_t h[32];
      if (((q.meta >> 8) & 0xffu) != ST_DECODE_FAILED) {
        wire_sighash(m, h);
      } else {
#pragma unroll
        for (int k = 0; k < 32; ++k) h[k] = 0;
      }
      BFLAG_SET(BF_STAGE_FREE);
      if (prm.wire_sighash && live) {  // zeros for an undecodable item, as tx_rows_kernel
        const bool dec = ((q.meta >> 8) & 0xffu) != ST_DECODE_FAILED;
        uint32_t* dst = reinterpret_cast<uint32_t*>(prm.wire_sighash + (size_t)idx * 32);
#pragma unroll
        for (int k = 0; k < 8; ++k)
          dst[k] = dec ? (uint32_t)h[4 * k] | ((uint32_t)h[4 * k + 1] << 8) | ((uint32_t)h[4 * k + 2] << 16) |
                             ((uint32_t)h[4 * k + 3] << 24)
                       : 0u;
      }
      uint32_t zl[8];
      limbs_from_be32(zl, h);
      bool ovz;
      q.Z = sc_from_limbs(zl, ovz);  // msg mod n (main_impl.h:183)
      st_.mark(5);
    }
    const sc u1 = VERIFY ? sc_mul(rinv, q.Z) : sc_neg(sc_mul(rinv, q.Z));  // main_impl.h:114-117
    ge Rp;
    bool yok;
    if (VERIFY && __all(vc65 || !pok)) {  // every key of the wave uncompressed: no root (wave-uniform)
      Rp.y = fe_from_u256(vpy);
      yok = true;
    } else {
      yok = ge_set_xo(Rp, x, VERIFY ? vodd : pok && (q.recid & 1u) != 0);  // ge_set_xo_var, group_impl.h:216-237
    }
    if (VERIFY && vc65) {  // a 65-byte key: its own y, on the curve (eckey_impl.h:17-34)
      const fe yk = fe_from_u256(vpy);
      const fe cx = fe_add(fe_mul(fe_sqr(x), x), fe_from_u32(7));
      yok = fe_equal(cx, fe_sqr(yk));
      Rp.y = yk;
    }
    lds_put_fe<FE_LIMBS>(S.y, Rp.y.v, l);
    S.yok[l] = yok ? 1u : 0u;
    BFLAG_SET(BF_Y);
    st_.mark(3);
    const uint32_t* gcomb = prm.gtab + (size_t)2 * GTAB * PT_WORDS;
    gej Ga;
    bool ginf;
    comb_mid<false>(Ga, ginf, u1, gcomb, dg);
    if (dg.force || __any(!ginf && fe_is_zero(Ga.z))) {
      diag_bump(dg, EGES_DIAG_MID_REDO);
      comb_mid<true>(Ga, ginf, u1, gcomb, dg);
    }
    // part[0] shares LDS with the wire stage: wave X reads its R from the stage (wire_r_only) before
    // it publishes its first point, so that count is the stage's release for this write (wave S's
    // own reads end at BF_STAGE_FREE; part[1] is written after BF_A1, i.e. after X's whole chain)
    if (wire) CNT_WAIT(BF_PUB, 1u);
    rg.part_put(0, Ga, l);
    S.pinf[0][l] = ginf ? 1u : 0u;
    BFLAG_SET(BF_G);
    st_.mark(4);
    stamp_out();
    return;
  }
  // R' = (c x, c^2) on E': y^2 = x^3 + 7 c^3, c = x^3 + 7 (no square root on this path)
  const fe c = fe_normalize_weak(fe_add(fe_mul(fe_sqr(x), x), fe_from_u32(7)));
  if (wv == 0) {  // ---- X: the doubling chain
    st_.mark(0);
    gej P;
    P.x = fe_mul(c, x);
    P.y = fe_sqr(c);
    P.z = fe_one();
    uint32_t freed = BK_RING;  // slots known free: points < freed - BK_RING consumed by both halves
#pragma unroll 1
    for (int k = 0; k < BK_WIN; ++k) {
      if (k > 0) {
#pragma unroll 1
        for (int i = 0; i < BK_BITS; ++i) P = gej_double(P);  // R' has odd order: never exceptional
      }
      if ((uint32_t)k >= freed) {  // slot k % BK_RING is free once both halves consumed point k - BK_RING
        st_.mark(1);
        CNT_WAIT(BF_CON0, (uint32_t)(k - BK_RING + 1));
        CNT_WAIT(BF_CON1, (uint32_t)(k - BK_RING + 1));
        const uint32_t c0 = ho_load(&S.flag[BF_CON0]), c1 = ho_load(&S.flag[BF_CON1]);
        freed = (c0 < c1 ? c0 : c1) + BK_RING;
        st_.mark(2);
      }
      rg.ring_put((uint32_t)(k % BK_RING), P, l);
      CNT_SET(BF_PUB, (uint32_t)(k + 1));
    }
    st_.mark(1);
    // then, per half, B1 + B3 of its final buckets (the halves' own waves do the rest of the sum
    // meanwhile), into a drained ring slot
#pragma unroll 1
    for (int h = 0; h < 2; ++h) {
      BFLAG_WAIT(BF_FIN0 + h);
      const uint32_t slot = (uint32_t)(BK_ASLOT + h), pt = slot + (uint32_t)BK_RING * ((BK_WIN - 1 - slot) / BK_RING);
      CNT_WAIT(BF_CON0, pt + 1);  // the last point that slot held, consumed by both halves
      CNT_WAIT(BF_CON1, pt + 1);
      bool ia;
      const gej a = join_mid(lds_get_gej(S.bucket[h][0], l), S.binf[h][0][l] != 0, lds_get_gej(S.bucket[h][2], l),
                             S.binf[h][2][l] != 0, ia, dg);
      rg.ring_put(slot, a, l);
      S.ainf[h][l] = ia ? 1u : 0u;
      BFLAG_SET(BF_A0 + h);
    }
    st_.mark(2);
    stamp_out();
    return;
  }
  // ---- Y1 / Y2: the buckets of one GLV half
  const int h = (int)wv - 2;
  st_.mark(0);
#pragma unroll
  for (int v = 0; v < BK_NB; ++v) S.binf[h][v][l] = 1u;
  BFLAG_WAIT(BF_DIG);
  st_.mark(1);
  uint32_t avail = 0;  // points known published
#pragma unroll 1
  for (int k = 0; k < BK_WIN; ++k) {
    if ((uint32_t)k >= avail) {
      st_.mark(2);
      CNT_WAIT(BF_PUB, (uint32_t)(k + 1));
      avail = ho_load(&S.flag[BF_PUB]);
      st_.mark(3);
    }
    gej P = rg.ring_get((uint32_t)(k % BK_RING), l);
    const int d = (int)S.dig[h][k][l];
    CNT_SET(BF_CON0 + h, (uint32_t)(k + 1));  // (the release fence orders this wave's ring reads first)
    const int a = d < 0 ? -d : d;
    const int v = a > 0 ? a - 1 : 0;
    P.y = fe_select(d < 0, fe_neg<1>(P.y), P.y);
    const gej B = lds_get_gej(S.bucket[h][v], l);
    const bool binf = S.binf[h][v][l] != 0;
    const gej s = gej_select(binf, P, gej_add_fast(B, P));
    if (d != 0) {
      lds_put_gej(S.bucket[h][v], s, l);
      S.binf[h][v][l] = 0u;
    }
  }
  st_.mark(2);
  // Q_h = B1 + 2 B2 + 3 B3 + 4 B4 = (B1 + B3) + 2 ((B2 + B3) + 2 B4): wave X joins B1 + B3
  // (its chain is done), this wave the rest: three joins and two doublings on this path
  static_assert(BK_NB == 4, "bucket sum written for 3-bit windows");
  BFLAG_SET(BF_FIN0 + h);
  bool ib, tinf;
  const bool i3 = S.binf[h][2][l] != 0;
  gej Jb = join_mid(lds_get_gej(S.bucket[h][1], l), S.binf[h][1][l] != 0, lds_get_gej(S.bucket[h][2], l), i3, ib, dg);
  Jb = join_mid(Jb, ib, gej_double(lds_get_gej(S.bucket[h][3], l)), S.binf[h][3][l] != 0, ib, dg);
  Jb = gej_double(Jb);
  BFLAG_WAIT(BF_A0 + h);
  gej T = join_mid(rg.ring_get((uint32_t)(BK_ASLOT + h), l), S.ainf[h][l] != 0, Jb, ib, tinf, dg);
  st_.mark(4);
  if (h == 1) {
    T.x = fe_mul(T.x, fe_const(FE_BETA));  // lambda (X, Y, Z) = (beta X, Y, Z)
    if (wire) BFLAG_WAIT(BF_STAGE_FREE);  // part[1] shares LDS with the stage
    rg.part_put(1, T, l);
    S.pinf[1][l] = tinf ? 1u : 0u;
    BFLAG_SET(BF_Q2);
    stamp_out();
    return;
  }
  // ---- Y1: the joins and the address
  BFLAG_WAIT(BF_Q2);
  bool qinf, oinf;
  gej Q = join_mid(T, tinf, rg.part_get(1, l), S.pinf[1][l] != 0, qinf, dg);
  BFLAG_WAIT(BF_Y);
  fe y;
  lds_get_fe<FE_LIMBS>(S.y, y.v, l);
  const bool yok = S.yok[l] != 0;
  Q.z = fe_mul(Q.z, y);  // E' -> E: (X, Y, Z) is (X, Y, Z y)
  BFLAG_WAIT(BF_G);
  st_.mark(5);
  Q = join_mid(Q, qinf, rg.part_get(0, l), S.pinf[0][l] != 0, oinf, dg);
  qinf = oinf;
  if (wire) {
    BFLAG_WAIT(BF_PARSED);
    q.meta = S.meta[l];
  }
  const bool fault = ho_failed(&S.flag[BF_ERR], dg);  // after Y1's last wait
  const bool ok = (wire ? S.pok[l] != 0 : pok) && yok && !qinf && !fault;  // main_impl.h:120
  if constexpr (VERIFY) {
    // x(Q) mod n == r  <=>  r Z^2 == X  or  (r < p - n and (r + n) Z^2 == X)  (ecdsa_impl.h:246-270)
    const fe z2 = fe_sqr(Q.z);
    bool eq = fe_equal(Q.x, fe_mul(fe_from_u256(q.R.v), z2));
    uint32_t rn[8];
    uint64_t cy = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      cy += (uint64_t)q.R.v[k] + SC_N[k];
      rn[k] = (uint32_t)cy;
      cy >>= 32;
    }
    eq = eq || (!u256_ge(q.R.v, P_MINUS_N) && fe_equal(Q.x, fe_mul(fe_from_u256(rn), z2)));
    if (live) {  // ok stays 0 / 1 (eges.h): a faulted item reads invalid, the fault word says why
      prm.v_ok[idx] = (!fault && ok && eq) ? 1 : 0;
      if (fault && prm.v_fault) __hip_atomic_store(prm.v_fault, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    st_.mark(7);
    stamp_out();
    return;
  }
  if (__any(ok && fe_is_zero(Q.z))) diag_bump(dg, EGES_DIAG_MID_EXC);  // never (see above)
  st_.mark(5);
  const fe zq = fe_select(ok && !fe_is_zero(Q.z), Q.z, fe_one());  // (see recover_mid_body)
  const fe zi = fe_inv_wave(zq);
  const fe zi2 = fe_sqr(zi);
  uint32_t X[8], Y[8];
  fe_to_u256(X, fe_normalize(fe_mul(Q.x, zi2)));
  fe_to_u256(Y, fe_normalize(fe_mul(Q.y, fe_mul(zi2, zi))));
  st_.mark(6);
  if (live) {
    const uint32_t pre_st = (q.meta >> 8) & 0xffu;
    prm.status[idx] = (uint8_t)(fault ? ST_ENGINE_FAULT : pre_st != ST_OK ? pre_st : (ok ? ST_OK : ST_RECOVER_FAILED));
    if (prm.addr) {
      uint32_t a[5];
      pub_address(a, X, Y);
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
  }
  st_.mark(7);
  stamp_out();
}

__global__ void __launch_bounds__(MID_WG, 1) recover_bkt_kernel(RecoverParams prm) {
  recover_bkt_body<NoStamp>(prm, nullptr);
}

__global__ void __launch_bounds__(MID_WG, 1) verify_bkt_kernel(RecoverParams prm) {
  recover_bkt_body<NoStamp, true>(prm, nullptr);
}
// two workgroups per CU (ring and parts in the workspace, no wire form)
__global__ void __launch_bounds__(MID_WG, 2) recover_bkt2_kernel(RecoverParams prm) {
  recover_bkt_body<NoStamp, false, true>(prm, nullptr);
}
__global__ void __launch_bounds__(MID_WG, 2) verify_bkt2_kernel(RecoverParams prm) {
  recover_bkt_body<NoStamp, true, true>(prm, nullptr);
}
size_t bkt2_ws_bytes_per_block() { return BK2_WS_WORDS * sizeof(uint32_t); }

__global__ void __launch_bounds__(MID_WG, 2) recover_mid_kernel(RecoverParams prm) {
  recover_mid_body<NoStamp>(prm, nullptr);
}

size_t mid_ws_bytes_per_block() { return MID_WS_WORDS * sizeof(uint32_t); }

hipError_t launch_verify_mid(const VerifyParams& v, bool two, size_t ws_bytes, hipStream_t st) {
  if (v.n == 0) return hipSuccess;
  const uint32_t grid = (v.n + MID_L - 1) / MID_L;
  if (two && (!v.ws || (size_t)grid * bkt2_ws_bytes_per_block() > ws_bytes)) return hipErrorInvalidValue;
  RecoverParams p{nullptr, v.n, v.n, nullptr, nullptr, nullptr, v.gtab, two ? v.ws : nullptr};
  p.diag = v.diag;
  p.force_redo = v.force_redo;
  p.test_skip_flag = v.test_skip_flag;
  p.test_skip_block = v.test_skip_block;
  p.v_pub = v.pub;
  p.v_publen = v.publen;
  p.v_msg = v.msg;
  p.v_sig = v.sig;
  p.v_ok = v.ok;
  p.v_fault = v.fault;
  if (two) hipLaunchKernelGGL(verify_bkt2_kernel, dim3(grid), dim3(MID_WG), 0, st, p);
  else hipLaunchKernelGGL(verify_bkt_kernel, dim3(grid), dim3(MID_WG), 0, st, p);
  return hipGetLastError();
}
// the two-per-CU bucket form: ws holds ceil(n / 64) blocks of bkt2_ws_bytes_per_block(); no wire form
hipError_t launch_recover_bkt2(const RecoverParams& p, size_t ws_bytes, hipStream_t st) {
  if (p.n == 0) return hipSuccess;
  const uint32_t grid = (p.n + MID_L - 1) / MID_L;
  if (p.wire_raw || !p.ws || (size_t)grid * bkt2_ws_bytes_per_block() > ws_bytes) return hipErrorInvalidValue;
  hipLaunchKernelGGL(recover_bkt2_kernel, dim3(grid), dim3(MID_WG), 0, st, p);
  return hipGetLastError();
}

// ws must hold ceil(n / 64) blocks of mid_ws_bytes_per_block(); the caller checks
hipError_t launch_recover_mid(const RecoverParams& p, bool bucket, size_t ws_bytes, hipStream_t st) {
  if (p.n == 0) return hipSuccess;
  if (bucket) {  // no workspace
    hipLaunchKernelGGL(recover_bkt_kernel, dim3((p.n + MID_L - 1) / MID_L), dim3(MID_WG), 0, st, p);
    return hipGetLastError();
  }
  const uint32_t grid = (p.n + MID_L - 1) / MID_L;
  if ((size_t)grid * mid_ws_bytes_per_block() > ws_bytes) return hipErrorInvalidValue;
  hipLaunchKernelGGL(recover_mid_kernel, dim3(grid), dim3(MID_WG), 0, st, p);
  return hipGetLastError();
}

#ifdef EGES_PHASE_STAMPS
__global__ void __launch_bounds__(MID_WG, 2) recover_mid_kernel_stamped(RecoverParams prm, uint64_t* stamps) {
  recover_mid_body<Stamper>(prm, stamps);
}
__global__ void __launch_bounds__(MID_WG, 1) recover_bkt_kernel_stamped(RecoverParams prm, uint64_t* stamps) {
  recover_bkt_body<Stamper>(prm, stamps);
}
hipError_t launch_recover_mid_stamped(const RecoverParams& p, bool bucket, size_t ws_bytes, hipStream_t st,
                                      uint64_t* stamps) {
  if (p.n == 0) return hipSuccess;
  if (bucket) {
    hipLaunchKernelGGL(recover_bkt_kernel_stamped, dim3((p.n + MID_L - 1) / MID_L), dim3(MID_WG), 0, st, p, stamps);
    return hipGetLastError();
  }
  const uint32_t grid = (p.n + MID_L - 1) / MID_L;
  if ((size_t)grid * mid_ws_bytes_per_block() > ws_bytes) return hipErrorInvalidValue;
  hipLaunchKernelGGL(recover_mid_kernel_stamped, dim3(grid), dim3(MID_WG), 0, st, p, stamps);
  return hipGetLastError();
}
#endif

}  // namespace eges
