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

namespace eges {

constexpr int MID_WG = 256;  // four waves
constexpr int MID_L = 64;    // signatures per workgroup (one per lane)
#ifndef EGES_MID_W0
#define EGES_MID_W0 15
#endif
constexpr int MID_W0 = EGES_MID_W0;  // windows [0, MID_W0) on wave A, the rest on waves B / C
constexpr int MID_HBITS = 4;
constexpr int MID_HTAB = 1 << (MID_HBITS - 1);
constexpr int MID_HWIN = (130 - RBITS * MID_W0 + MID_HBITS) / MID_HBITS;
static_assert(MID_W0 * RBITS + MID_HWIN * MID_HBITS >= 130, "windows cover a GLV half + carry");

enum { MF_DIG = 0, MF_Y, MF_G, MF_HB, MF_HC, MF_N };

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

DEV void mflag_set(uint32_t* f) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  if ((threadIdx.x & 63) == 0) __hip_atomic_store(f, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// Every producer sets its flags unconditionally; the bound (~1 s) only keeps a logic error from
// hanging the device (the results would then be wrong, and the tests say so).
DEV void mflag_wait(uint32_t* f) {
#pragma unroll 1
  for (uint32_t it = 0; it < (1u << 24); ++it) {
    if (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != 0u) break;
    __builtin_amdgcn_s_sleep(2);
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

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
  __shared__ MidLds S;
  ST st_;
  const Diag dg = diag_of(prm);
  const uint32_t l = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint32_t idx = blockIdx.x * MID_L + l;
  const bool live = idx < prm.n;
  if (threadIdx.x < MF_N) S.flag[threadIdx.x] = 0u;
  __syncthreads();  // the only barrier
  const LatParse q = lat_parse(prm, live ? idx : prm.n - 1);
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
    mflag_set(&S.flag[MF_DIG]);
    st_.mark(2);
    ge Rp;
    const bool yok = ge_set_xo(Rp, x, pok && (q.recid & 1u) != 0);  // ge_set_xo_var, group_impl.h:216-237
    lds_put_fe<FE_LIMBS>(S.y, Rp.y.v, l);
    S.yok[l] = yok ? 1u : 0u;
    mflag_set(&S.flag[MF_Y]);
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
    mflag_set(&S.flag[MF_G]);
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
    mflag_wait(&S.flag[MF_DIG]);
    st_.mark(3);
    gej H;
    bool hinf;
    if (j == 0) strauss_mid_exact<MID_HBITS, MID_HTAB, MID_HWIN, 1>(H, hinf, tab, S.hi[0], S.hi[1], l, dg);
    else strauss_mid_exact<MID_HBITS, MID_HTAB, MID_HWIN, 2>(H, hinf, tab, S.hi[0], S.hi[1], l, dg);
    H.z = fe_mul(H.z, scale);  // E' coordinates
    put_part_ls(S, 1 + j, H, hinf, l);
    mflag_set(&S.flag[j ? MF_HC : MF_HB]);
    st_.mark(4);
    stamp_out();
    return;
  }
  // ---- A: the R' table, the low windows of both halves, then the joins and the address
  uint32_t* tab = ws + MID_TAB_A;
  st_.mark(0);
  const fe zeta = build_table_mid<PTAB>(tab, ws + MID_ZR_A, Rp, l);
  st_.mark(3);
  mflag_wait(&S.flag[MF_DIG]);
  st_.mark(1);
  gej A;
  bool ainf;
  strauss_mid_exact<RBITS, PTAB, MID_W0, 3>(A, ainf, tab, S.lo[0], S.lo[1], l, dg);
  st_.mark(4);
  // back to E: an E' Jacobian point (X, Y, Z) is (X, Y, Z y) on E; the table curve adds zeta.
  // A + u1 G first (both are usually ready before the high waves finish), then the high parts.
  mflag_wait(&S.flag[MF_Y]);
  fe y;
  lds_get_fe<FE_LIMBS>(S.y, y.v, l);
  const bool yok = S.yok[l] != 0;
  A.z = fe_mul(A.z, fe_mul(zeta, y));
  bool binf, cinf, ginf, hinf, qinf;
  mflag_wait(&S.flag[MF_G]);
  st_.mark(7);
  const gej Gp = get_part_ls(S, 0, ginf, l);
  gej Q = join_mid(A, ainf, Gp, ginf, qinf, dg);
  st_.mark(2);
  mflag_wait(&S.flag[MF_HB]);
  mflag_wait(&S.flag[MF_HC]);
  st_.mark(7);
  gej Hb = get_part_ls(S, 1, binf, l), Hc = get_part_ls(S, 2, cinf, l);
  Hb.z = fe_mul(Hb.z, y);
  Hc.z = fe_mul(Hc.z, y);
  const gej H = join_mid(Hb, binf, Hc, cinf, hinf, dg);
  Q = join_mid(Q, qinf, H, hinf, qinf, dg);
  st_.mark(2);
  const bool ok = pok && yok && !qinf;  // main_impl.h:120
  // affine, serialize, address
  const fe zi = fe_inv(fe_select(ok, Q.z, fe_one()));
  const fe zi2 = fe_sqr(zi);
  uint32_t X[8], Y[8];
  fe_to_u256(X, fe_normalize(fe_mul(Q.x, zi2)));
  fe_to_u256(Y, fe_normalize(fe_mul(Q.y, fe_mul(zi2, zi))));
  st_.mark(5);
  if (live) {
    const uint32_t pre_st = (q.meta >> 8) & 0xffu;
    prm.status[idx] = (uint8_t)(pre_st != ST_OK ? pre_st : (ok ? ST_OK : ST_RECOVER_FAILED));
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

__global__ void __launch_bounds__(MID_WG, 2) recover_mid_kernel(RecoverParams prm) {
  recover_mid_body<NoStamp>(prm, nullptr);
}

size_t mid_ws_bytes_per_block() { return MID_WS_WORDS * sizeof(uint32_t); }

// ws must hold ceil(n / 64) blocks of mid_ws_bytes_per_block(); the caller checks
hipError_t launch_recover_mid(const RecoverParams& p, size_t ws_bytes, hipStream_t st) {
  if (p.n == 0) return hipSuccess;
  const uint32_t grid = (p.n + MID_L - 1) / MID_L;
  if ((size_t)grid * mid_ws_bytes_per_block() > ws_bytes) return hipErrorInvalidValue;
  hipLaunchKernelGGL(recover_mid_kernel, dim3(grid), dim3(MID_WG), 0, st, p);
  return hipGetLastError();
}

#ifdef EGES_PHASE_STAMPS
__global__ void __launch_bounds__(MID_WG, 2) recover_mid_kernel_stamped(RecoverParams prm, uint64_t* stamps) {
  recover_mid_body<Stamper>(prm, stamps);
}
hipError_t launch_recover_mid_stamped(const RecoverParams& p, size_t ws_bytes, hipStream_t st, uint64_t* stamps) {
  if (p.n == 0) return hipSuccess;
  const uint32_t grid = (p.n + MID_L - 1) / MID_L;
  if ((size_t)grid * mid_ws_bytes_per_block() > ws_bytes) return hipErrorInvalidValue;
  hipLaunchKernelGGL(recover_mid_kernel_stamped, dim3(grid), dim3(MID_WG), 0, st, p, stamps);
  return hipGetLastError();
}
#endif

}  // namespace eges
