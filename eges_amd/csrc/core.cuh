#pragma once
// Shared device core of the secp256k1 sender-recovery kernels (gfx950).
//
// Hot path: for every signature record
//   parse (r, s, recid) ........... recovery/main_impl.h:38-58 (overflow => failure)
//   x = r (+ n if recid & 2) ...... main_impl.h:101-109
//   R = lift_x(x, recid & 1) ...... group_impl.h:216-237 via (p+1)/4 sqrt, field_impl.h:38-134
//   r^-1 mod n .................... scalar_impl.h:262-281 -> per-thread Montgomery batch inversion
//   u1 = -z/r, u2 = s/r ........... main_impl.h:114-117 (z = msg mod n, :183)
//   Q = u2*R + u1*G ............... ecmult_impl.h:286-404 -> GLV split of u2 + 5-bit signed
//                                   windows for R / lambda*R (per-lane 16-entry table on one
//                                   global Z, built with co-Z additions); u1 split at 2^128 with
//                                   20-bit signed windows against {1..2^19}*G and *2^128*G
//   Q == infinity => failure ...... main_impl.h:120
//   affine (batch inversion), serialize 04||X||Y (eckey_impl.h:36-52), Keccak-256 address
//                                   (crypto.go:194-197, transaction_signing.go:245)
//
// Execution model: see k_recover.hip (lane-serial batches, one thread per signature stream).
// All control flow that depends on data is either per-lane selects or wave-uniform (ballot)
// branches for the rare exceptional additions.
#include <type_traits>

#include "fe.cuh"
#include "sc.cuh"
#include "ge.cuh"
#include "keccak.cuh"
#include "launch.h"
#include "eges.h"  // EGES_DIAG_* counter indices

namespace eges {

constexpr int WG = 256;
constexpr int NWAVES = WG / 64;
// R / lambda R: signed windows of RBITS bits over a GLV half (|k| < 2^129, plus one bit for
// the recoding carry) against the per-lane table {1..2^(RBITS-1)}*R.
constexpr int RBITS = 5;
constexpr int RWIN = (130 + RBITS - 1) / RBITS;  // 26 windows of 5 bits (33 of 4)
constexpr int PTAB = 1 << (RBITS - 1);           // {1..16}*R per lane
// Fixed base: u_g = lo + 2^128 hi (libsecp's split_128, ecmult_impl.h:349), signed windows of
// GBITS bits over each 128-bit half against the tables {1..GTAB}*G and {1..GTAB}*2^128*G.
constexpr int GBITS = 20;                 // multiple of RBITS: aligned with the R windows
constexpr int GSTEP = GBITS / RBITS;              // R windows per G window
constexpr int GWIN = (RWIN + GSTEP - 1) / GSTEP;  // G windows
constexpr int GTAB = 1 << (GBITS - 1);
// Comb table of the latency kernels (after the two GTAB tables in the same allocation):
// entry (k, i) = (i + 1) 2^(16 k) G, k < 16, i < 2^16 - 1, so u G = sum_k T_k[digit_k - 1] over
// the 16 unsigned 16-bit digits of u: 16 additions and no doublings.
constexpr int CBITS = 16, CWIN = 16, CTAB = (1 << CBITS) - 1;
static_assert(GBITS % RBITS == 0 && GWIN * GBITS >= 129, "G windows must cover a 128-bit half + carry");
using gdig_t = std::conditional_t<(GBITS > 16), int32_t, int16_t>;

enum : uint32_t {
  ST_OK = 0, ST_INVALID_CHAIN_ID = 1, ST_INVALID_SIG = 2, ST_INVALID_RECOVERY_ID = 5, ST_RECOVER_FAILED = 6,
  ST_DECODE_FAILED = 7, ST_ENGINE_FAULT = 0xFF
};

__constant__ const uint32_t FE_BETA[8] = {0x719501EEu, 0xC1396C28u, 0x12F58995u, 0x9CF04975u,
                                          0xAC3434E9u, 0x6E64479Eu, 0x657C0710u, 0x7AE96A2Bu};
__constant__ const uint32_t GEN_X[8] = {0x16F81798u, 0x59F2815Bu, 0x2DCE28D9u, 0x029BFCDBu,
                                        0xCE870B07u, 0x55A06295u, 0xF9DCBBACu, 0x79BE667Eu};
__constant__ const uint32_t GEN_Y[8] = {0xFB10D4B8u, 0x9C47D08Fu, 0xA6855419u, 0xFD17B448u,
                                        0x0E1108A8u, 0x5DA4FBFCu, 0x26A3C465u, 0x483ADA77u};
// 2^128 * G (second fixed-base table)
__constant__ const uint32_t G128_X[8] = {0x9EC4C0DAu, 0x1B7B444Cu, 0x723EA335u, 0xE88C5678u,
                                         0x981F162Eu, 0x9239C1ADu, 0xF63B5F33u, 0x8F68B9D2u};
__constant__ const uint32_t G128_Y[8] = {0x501FFF82u, 0xF23CBF79u, 0x95510BFDu, 0xBBEA2CFEu,
                                         0xB6BE215Du, 0xDE1D90C2u, 0xBA063986u, 0x662A9F2Du};
// p, little-endian 32-bit limbs (field_10x26_impl.h set_b32 rejects >= p)
__constant__ const uint32_t FE_P[8] = {0xFFFFFC2Fu, 0xFFFFFFFEu, 0xFFFFFFFFu, 0xFFFFFFFFu,
                                       0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
// p - n  (recovery/main_impl.h:104, ecdsa_impl.h:45-47)
__constant__ const uint32_t P_MINUS_N[8] = {0x2FC9BAEEu, 0x402DA172u, 0x50B75FC4u, 0x45512319u,
                                            0x00000001u, 0u, 0u, 0u};

DEV fe fe_const(const uint32_t* c) { return fe_from_u256(c); }

template <class T>
constexpr int NL = sizeof(T) / sizeof(uint32_t);  // limbs of fe (9) / sc (8)
DEV ge gen_point() {
  ge g;
  g.x = fe_const(GEN_X);
  g.y = fe_const(GEN_Y);
  return g;
}

// ------------------------------------------------------------------ diagnostics
// Where a kernel's rare exact branches report (EGES_DIAG_*, eges_diag_counters) and whether a
// test forces every exact-redo pass (KNOB_FORCE_REDO). Both wave-uniform.
struct Diag {
  uint32_t* ctr = nullptr;
  bool force = false;
};
// one increment per wave: the first active lane adds (a vector-memory atomic)
DEV void diag_bump(const Diag& d, int k) {
  if (!d.ctr) return;
  const uint64_t act = __ballot(1);
  if ((uint32_t)__lane_id() == (uint32_t)__builtin_ctzll(act))
    __hip_atomic_fetch_add(d.ctr + k, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <class P>
DEV Diag diag_of(const P& prm) {
  Diag d;
  d.ctr = prm.diag;
  d.force = prm.force_redo != 0;
  return d;
}

// ------------------------------------------------------------------ cross-lane helpers
template <class T>
DEV T shfl_up_t(const T& x, int d) {
  T r;
#pragma unroll
  for (int i = 0; i < NL<T>; ++i) r.v[i] = (uint32_t)__shfl_up((int)x.v[i], d, 64);
  return r;
}
template <class T>
DEV T shfl_down_t(const T& x, int d) {
  T r;
#pragma unroll
  for (int i = 0; i < NL<T>; ++i) r.v[i] = (uint32_t)__shfl_down((int)x.v[i], d, 64);
  return r;
}

struct FieldOps {
  using T = fe;
  static DEV T one() { return fe_one(); }
  static DEV T mul(const T& a, const T& b) { return fe_mul(a, b); }
  static DEV T inv(const T& a) { return fe_inv(a); }
  static DEV T sel(bool c, const T& a, const T& b) { return fe_select(c, a, b); }
};
struct ScalarOps {
  using T = sc;
  static DEV T one() { return sc_one(); }
  static DEV T mul(const T& a, const T& b) { return sc_mul(a, b); }
  static DEV T inv(const T& a) { return sc_inv(a); }
  static DEV T sel(bool c, const T& a, const T& b) { return sc_select(c, a, b); }
};

// Workgroup Montgomery batch inversion: returns a^-1 for valid lanes (garbage otherwise).
// Invalid lanes contribute 1 to the products so they cannot poison the batch.
// lds: at least 2 * NWAVES * 10 words (NL <= 10). Every thread of the workgroup must call this.
template <class Ops>
DEV typename Ops::T wg_batch_inv(const typename Ops::T& a, bool valid, uint32_t* lds) {
  using T = typename Ops::T;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  T x = Ops::sel(valid, a, Ops::one());
  T P = x;  // inclusive prefix product within the wave
#pragma unroll 1
  for (int d = 1; d < 64; d <<= 1) {
    T y = shfl_up_t(P, d);
    T m = Ops::mul(P, y);
    P = Ops::sel(lane >= d, m, P);
  }
  T Q = x;  // inclusive suffix product
#pragma unroll 1
  for (int d = 1; d < 64; d <<= 1) {
    T y = shfl_down_t(Q, d);
    T m = Ops::mul(Q, y);
    Q = Ops::sel(lane + d < 64, m, Q);
  }
  T pex = Ops::sel(lane == 0, Ops::one(), shfl_up_t(P, 1));
  T sex = Ops::sel(lane == 63, Ops::one(), shfl_down_t(Q, 1));
  if (lane == 63) {
#pragma unroll
    for (int i = 0; i < NL<T>; ++i) lds[wave * 10 + i] = P.v[i];
  }
  __syncthreads();
  if (wave == 0) {
    T t[NWAVES];
#pragma unroll
    for (int w = 0; w < NWAVES; ++w)
#pragma unroll
      for (int i = 0; i < NL<T>; ++i) t[w].v[i] = lds[w * 10 + i];
    T tot = t[0];
#pragma unroll
    for (int w = 1; w < NWAVES; ++w) tot = Ops::mul(tot, t[w]);
    T inv = Ops::inv(tot);
    const int me = lane & (NWAVES - 1);
#pragma unroll
    for (int w = 0; w < NWAVES; ++w) inv = Ops::mul(inv, Ops::sel(w == me, Ops::one(), t[w]));
    if (lane < NWAVES) {
#pragma unroll
      for (int i = 0; i < NL<T>; ++i) lds[NWAVES * 10 + lane * 10 + i] = inv.v[i];
    }
  }
  __syncthreads();
  T winv;
#pragma unroll
  for (int i = 0; i < NL<T>; ++i) winv.v[i] = lds[NWAVES * 10 + wave * 10 + i];
  __syncthreads();  // lds is reused by the next call
  return Ops::mul(Ops::mul(winv, pex), sex);
}

// ------------------------------------------------------------------ digit recoding
// Signed fixed-window recoding of a GLV half (|k| < 2^129) into NW digits of W bits,
// digits in [-(2^(W-1) - 1), 2^(W-1)] (table entries 1..2^(W-1)), the half's sign folded in.
// Written to LDS [w][WG]. NW * W >= 130 leaves no carry out of the top window.
template <int W, int NW, class D>
DEV void recode(const glv_half& h, D* out /* [NW][WG] */) {
  uint32_t m[5];
#pragma unroll
  for (int i = 0; i < 5; ++i) m[i] = h.mag[i];
  int carry = 0;
  const int tid = threadIdx.x;
#pragma unroll 1
  for (int w = 0; w < NW; ++w) {
    int v = (int)(m[0] & ((1u << W) - 1)) + carry;
    carry = v > (1 << (W - 1)) ? 1 : 0;
    v -= carry << W;
    out[w * WG + tid] = (D)(h.neg ? -v : v);
    // m >>= W
#pragma unroll
    for (int i = 0; i < 4; ++i) m[i] = (m[i] >> W) | (m[i + 1] << (32 - W));
    m[4] >>= W;
  }
}

// ------------------------------------------------------------------ tables
// Affine point record: x (9 radix-2^29 limbs), y (9 limbs), 2 words of padding: 80 bytes,
// 16-byte aligned, moved as five 16-byte accesses.
constexpr int PT_WORDS = 20;

DEV void pt_pack(uint32_t w[PT_WORDS], const fe& x, const fe& y) {
#pragma unroll
  for (int i = 0; i < FE_LIMBS; ++i) {
    w[i] = x.v[i];
    w[FE_LIMBS + i] = y.v[i];
  }
  w[18] = 0;
  w[19] = 0;
}
DEV void pt_unpack(const uint32_t w[PT_WORDS], fe& x, fe& y) {
#pragma unroll
  for (int i = 0; i < FE_LIMBS; ++i) {
    x.v[i] = w[i];
    y.v[i] = w[FE_LIMBS + i];
  }
}
DEV void store_pt(uint32_t* dst, const ge& p) {
  uint32_t w[PT_WORDS];
  pt_pack(w, p.x, p.y);
  uint4* d = reinterpret_cast<uint4*>(dst);
#pragma unroll
  for (int q = 0; q < 5; ++q) d[q] = make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
}
DEV ge load_pt(const uint32_t* src) {
  const uint4* s = reinterpret_cast<const uint4*>(src);
  uint32_t w[PT_WORDS];
#pragma unroll
  for (int q = 0; q < 5; ++q) {
    const uint4 u = s[q];
    w[4 * q] = u.x;
    w[4 * q + 1] = u.y;
    w[4 * q + 2] = u.z;
    w[4 * q + 3] = u.w;
  }
  ge p;
  pt_unpack(w, p.x, p.y);
  return p;
}

// ------------------------------------------------------------------ Strauss step
// acc += p when `use`; acc_inf tracks the point at infinity. Exceptional sums (acc == +-p)
// are resolved exactly on a wave-uniform slow path.
DEV void add_step(gej& acc, bool& inf, const ge& p, bool use, const Diag& dg, int slot = EGES_DIAG_LS_EXC) {
  bool hz, rz;
  gej s = gej_add_ge(acc, p, hz, rz);
  const bool exc = use && !inf && hz;
  if (__any(exc)) {
    diag_bump(dg, slot);
    gej d = gej_double(acc);
    s = gej_select(exc && rz, d, s);
  }
  const bool to_inf = exc && !rz;
  gej pj = gej_from_ge(p);
  gej nacc = gej_select(inf, pj, s);
  acc = gej_select(use, nacc, acc);
  inf = use ? (inf ? false : to_inf) : inf;
}

// acc (on the table's isomorphic curve, global Z = zeta) += p (affine on the true curve).
DEV void add_step_zinv(gej& acc, bool& inf, const ge& p, bool use, const fe& zeta, const Diag& dg) {
  bool hz, rz;
  gej s = gej_add_ge_zinv(acc, p, zeta, hz, rz);
  const bool exc = use && !inf && hz;
  if (__any(exc)) {
    diag_bump(dg, EGES_DIAG_LS_EXC);
    gej d = gej_double(acc);
    s = gej_select(exc && rz, d, s);
  }
  const bool to_inf = exc && !rz;
  if (__any(use && inf)) {  // acc = p mapped onto the isomorphic curve: (x zeta^2, y zeta^3, 1)
    const fe z2 = fe_sqr(zeta);
    gej pj;
    pj.x = fe_mul(p.x, z2);
    pj.y = fe_mul(p.y, fe_mul(z2, zeta));
    pj.z = fe_one();
    s = gej_select(inf, pj, s);
  }
  acc = gej_select(use, s, acc);
  inf = use ? (inf ? false : to_inf) : inf;
}

// Unchecked forms: an exceptional sum poisons acc (Z == 0, ge.cuh CHECK) instead of being
// resolved; ecmult_core detects that once per signature and redoes the lane exactly.
DEV void add_step_fast(gej& acc, bool& inf, const ge& p, bool use) {
  gej s = gej_add_ge_fast(acc, p);
  s = gej_select(inf, gej_from_ge(p), s);
  acc = gej_select(use, s, acc);
  inf = inf && !use;
}
DEV void add_step_zinv_fast(gej& acc, bool& inf, const ge& p, bool use, const fe& zeta) {
  gej s = gej_add_ge_zinv_fast(acc, p, zeta);
  if (__any(use && inf)) {
    const fe z2 = fe_sqr(zeta);
    gej pj;
    pj.x = fe_mul(p.x, z2);
    pj.y = fe_mul(p.y, fe_mul(z2, zeta));
    pj.z = fe_one();
    s = gej_select(inf, pj, s);
  }
  acc = gej_select(use, s, acc);
  inf = inf && !use;
}

DEV ge neg_if(const ge& p, bool neg) {  // y magnitude <= 2 afterwards
  ge r;
  r.x = p.x;
  r.y = fe_select(neg, fe_neg<1>(p.y), p.y);
  return r;
}

struct CoreLds {
  int8_t rdig[2][RWIN][WG];    // R / lambda R digits
  gdig_t gdig[2][GWIN][WG];    // G / 2^128 G digits
  uint32_t inv_scratch[2 * NWAVES * 10];
  uint32_t zeta[FE_LIMBS][WG];  // per-lane global Z of the R table
};

template <int N>
DEV void lds_put(uint32_t (*a)[WG], const uint32_t* v) {
#pragma unroll
  for (int i = 0; i < N; ++i) a[i][threadIdx.x] = v[i];
}
template <int N>
DEV void lds_get(uint32_t (*a)[WG], uint32_t* v) {
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] = a[i][threadIdx.x];
}

// Per-block workspace (global memory, this block's lanes only):
//   [0, PTAB*WG*PT_WORDS)              table {1..PTAB}*P, entry-major then lane
//   [ZR_OFF, +(PTAB-1)*WG*ZR_WORDS)    Z ratios Z_{i+1}/Z_i while the table is built
//   [PARK_OFF, +PARK_ROWS*WG)          per-thread registers parked across ecmult_core
constexpr int ZR_WORDS = 12;  // one field element, three 16-byte accesses
constexpr int PARK_ROWS = 18;
constexpr size_t ZR_OFF = (size_t)PTAB * WG * PT_WORDS;
constexpr size_t PARK_OFF = ZR_OFF + (size_t)(PTAB - 1) * WG * ZR_WORDS;
constexpr size_t WS_WORDS = PARK_OFF + (size_t)PARK_ROWS * WG;

// park / unpark N words of this thread at row offset r of the block's park area
template <int N>
DEV void park_put(uint32_t* ws, int r, const uint32_t* v) {
  uint32_t* a = ws + (size_t)blockIdx.x * WS_WORDS + PARK_OFF + (size_t)r * WG + threadIdx.x;
#pragma unroll
  for (int i = 0; i < N; ++i) a[(size_t)i * WG] = v[i];
}
template <int N>
DEV void park_get(const uint32_t* ws, int r, uint32_t* v) {
  const uint32_t* a = ws + (size_t)blockIdx.x * WS_WORDS + PARK_OFF + (size_t)r * WG + threadIdx.x;
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] = a[(size_t)i * WG];
}

DEV void store_fe2(uint32_t* dst, const fe& a, const fe& b) {
  ge p;
  p.x = a;
  p.y = b;
  store_pt(dst, p);
}
DEV void store_fe(uint32_t* dst, const fe& a) {
  uint4* d = reinterpret_cast<uint4*>(dst);
  d[0] = make_uint4(a.v[0], a.v[1], a.v[2], a.v[3]);
  d[1] = make_uint4(a.v[4], a.v[5], a.v[6], a.v[7]);
  d[2] = make_uint4(a.v[8], 0u, 0u, 0u);
}
DEV fe load_fe(const uint32_t* src) {
  const uint4* s = reinterpret_cast<const uint4*>(src);
  const uint4 a = s[0], b = s[1], c = s[2];
  fe r;
  r.v[0] = a.x; r.v[1] = a.y; r.v[2] = a.z; r.v[3] = a.w;
  r.v[4] = b.x; r.v[5] = b.y; r.v[6] = b.z; r.v[7] = b.w;
  r.v[8] = c.x;
  return r;
}

// Diagnostic phase stamps (EGES_PHASE_STAMPS builds only): per-wave s_memtime deltas.
struct NoStamp {
  DEV void mark(int) {}
};
struct Stamper {
  uint64_t acc[8];
  uint64_t last;
  DEV Stamper() {
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = 0;
    last = __builtin_amdgcn_s_memtime();
  }
  DEV void mark(int i) {
    const uint64_t now = __builtin_amdgcn_s_memtime();
    acc[i] += now - last;
    last = now;
  }
};


// Strauss-Shamir over the digits in L and the tables (per-lane R table at `base`, G / lambda G
// in gtab): acc = sum of the window contributions on the R table's isomorphic curve.
template <bool CHECKED>
DEV void strauss(gej& acc, bool& inf, const uint32_t* base, const uint32_t* gtab, CoreLds& L, const Diag& dg) {
  const int tid = threadIdx.x;
  // RWIN windows of RBITS bits (R, lambda R) interleaved with GWIN windows of GBITS bits
  // (G, 2^128 G) every GSTEP-th window.
  inf = true;
  acc.x = fe_zero();
  acc.y = fe_zero();
  acc.z = fe_zero();
#pragma unroll 1
  for (int w = RWIN - 1; w >= 0; --w) {
    if (w != RWIN - 1) {
#pragma unroll 1
      for (int k = 0; k < RBITS; ++k) acc = gej_double(acc);
    }
    const int nadd = (w % GSTEP) == 0 ? 4 : 2;
#pragma unroll 1
    for (int j = 0; j < nadd; ++j) {
      int d;
      if (j < 2) d = L.rdig[j][w][tid];
      else d = L.gdig[j - 2][w / GSTEP][tid];
      const int a = d < 0 ? -d : d;
      const int e = a > 0 ? a - 1 : 0;
      ge p;
      if (j < 2) p = load_pt(base + (size_t)(e * WG + tid) * PT_WORDS);
      else p = load_pt(gtab + ((size_t)(j - 2) * GTAB + e) * PT_WORDS);
      if (j == 1) p.x = fe_mul(p.x, fe_const(FE_BETA));
      if (j < 2) {
        if (CHECKED) add_step(acc, inf, neg_if(p, d < 0), d != 0, dg);
        else add_step_fast(acc, inf, neg_if(p, d < 0), d != 0);
      } else {
        fe z;
        lds_get<FE_LIMBS>(L.zeta, z.v);
        if (CHECKED) add_step_zinv(acc, inf, neg_if(p, d < 0), d != 0, z, dg);
        else add_step_zinv_fast(acc, inf, neg_if(p, d < 0), d != 0, z);
      }
    }
  }
}

// Q = u_r * P + u_g * G for the workgroup's 256 lanes. P given affine (a valid curve point,
// possibly a dummy for failed lanes). Returns Jacobian Q and its infinity flag.
template <class ST = NoStamp>
DEV void ecmult_core(gej& acc, bool& inf, const ge& P, const sc& u_r, const sc& u_g, const uint32_t* gtab,
                     uint32_t* ws, CoreLds& L, ST* st = nullptr, const Diag& dg = Diag()) {
  const int tid = threadIdx.x;
  uint32_t* const base = ws + (size_t)blockIdx.x * WS_WORDS;
  // --- digits
  {
    glv_half h1, h2;
    glv_split(h1, h2, u_r);
    recode<RBITS, RWIN, int8_t>(h1, &L.rdig[0][0][0]);
    recode<RBITS, RWIN, int8_t>(h2, &L.rdig[1][0][0]);
    glv_half g0, g1;  // u_g = lo + 2^128 hi, both non-negative
    g0.neg = false;
    g1.neg = false;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      g0.mag[i] = u_g.v[i];
      g1.mag[i] = u_g.v[4 + i];
    }
    g0.mag[4] = 0;
    g1.mag[4] = 0;
    recode<GBITS, GWIN, gdig_t>(g0, &L.gdig[0][0][0]);
    recode<GBITS, GWIN, gdig_t>(g1, &L.gdig[1][0][0]);
  }
  if (st) st->mark(2);
  // --- per-lane table {1..PTAB} * P with one global Z (the idea of ecmult_impl.h:52-110,
  //     built with co-Z additions): T_2 = 2P and P share Z_2 = 2y (gej_dblu); each
  //     T_{i+1} = T_i + P is a co-Z addition that also moves P onto the new Z (gej_zaddu),
  //     recording the ratios Z_{i+1}/Z_i. A backward pass rescales every T_i to
  //     Z_PTAB = zeta: the entries are affine points of the isomorphic curve
  //     y^2 = x^3 + 7 zeta^6 — no field inversion. T_i == +-P never happens for 1 < i < n.
  fe zeta;
  {
    store_pt(base + (size_t)tid * PT_WORDS, P);
    gej D;
    ge B;
    gej_dblu(D, B, P);
    store_fe(base + ZR_OFF + (size_t)tid * ZR_WORDS, D.z);  // Z_2 / Z_1 = 2y
    ge T;
    T.x = D.x;
    T.y = D.y;
    store_pt(base + (size_t)(1 * WG + tid) * PT_WORDS, T);
#pragma unroll 1
    for (int i = 2; i < PTAB; ++i) {
      const fe zr = gej_zaddu(T, B);  // T = (i+1) P
      store_pt(base + (size_t)(i * WG + tid) * PT_WORDS, T);
      store_fe(base + ZR_OFF + (size_t)((i - 1) * WG + tid) * ZR_WORDS, zr);
    }
    fe rho = fe_one();
#pragma unroll 1
    for (int i = PTAB - 2; i >= 0; --i) {
      const fe zr = load_fe(base + ZR_OFF + (size_t)(i * WG + tid) * ZR_WORDS);  // Z_{i+2} / Z_{i+1}
      rho = i == PTAB - 2 ? zr : fe_mul(rho, zr);                                // Z_PTAB / Z_{i+1}
      const ge J = load_pt(base + (size_t)(i * WG + tid) * PT_WORDS);
      const fe r2 = fe_sqr(rho);
      ge a;
      a.x = fe_mul(J.x, r2);
      a.y = fe_mul(J.y, fe_mul(r2, rho));
      store_pt(base + (size_t)(i * WG + tid) * PT_WORDS, a);
    }
    zeta = rho;  // Z_PTAB / Z_1 with Z_1 = 1
    lds_put<FE_LIMBS>(L.zeta, zeta.v);
  }
  if (st) st->mark(3);
  // --- Strauss-Shamir, unchecked; exact redo of the whole wave if any lane was poisoned
  strauss<false>(acc, inf, base, gtab, L, dg);
  if (dg.force || __any(!inf && fe_is_zero(acc.z))) {
    diag_bump(dg, EGES_DIAG_LS_REDO);
    strauss<true>(acc, inf, base, gtab, L, dg);
  }
  // true Jacobian Z of the accumulator
  {
    fe z;
    lds_get<FE_LIMBS>(L.zeta, z.v);
    acc.z = fe_mul(acc.z, z);
  }
  if (st) st->mark(4);
}

// ------------------------------------------------------------------ lane-serial kernels
// Per-item state between the phases of the recover / verify kernels lives in uint4 slot rows of
// n_pad entries (recover: 0-4 R then Q.x/Q.y, 5-6 prefix product of r, 7-11 Q.z and the prefix
// product of Z; verify: 0-4 P, 5-6 prefix product of s).
DEV void slot_put_pt(uint4* slot, uint32_t n_pad, int row, uint32_t idx, const ge& p) {
  uint32_t w[PT_WORDS];
  pt_pack(w, p.x, p.y);
#pragma unroll
  for (int q = 0; q < 5; ++q)
    slot[(size_t)(row + q) * n_pad + idx] = make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
}
DEV ge slot_get_pt(const uint4* slot, uint32_t n_pad, int row, uint32_t idx) {
  uint32_t w[PT_WORDS];
#pragma unroll
  for (int q = 0; q < 5; ++q) {
    const uint4 u = slot[(size_t)(row + q) * n_pad + idx];
    w[4 * q] = u.x;
    w[4 * q + 1] = u.y;
    w[4 * q + 2] = u.z;
    w[4 * q + 3] = u.w;
  }
  ge p;
  pt_unpack(w, p.x, p.y);
  return p;
}
DEV void slot_put_sc(uint4* slot, uint32_t n_pad, int row, uint32_t idx, const sc& a) {
  slot[(size_t)row * n_pad + idx] = make_uint4(a.v[0], a.v[1], a.v[2], a.v[3]);
  slot[(size_t)(row + 1) * n_pad + idx] = make_uint4(a.v[4], a.v[5], a.v[6], a.v[7]);
}
DEV sc slot_get_sc(const uint4* slot, uint32_t n_pad, int row, uint32_t idx) {
  const uint4 a = slot[(size_t)row * n_pad + idx], b = slot[(size_t)(row + 1) * n_pad + idx];
  sc r;
  r.v[0] = a.x; r.v[1] = a.y; r.v[2] = a.z; r.v[3] = a.w;
  r.v[4] = b.x; r.v[5] = b.y; r.v[6] = b.z; r.v[7] = b.w;
  return r;
}
DEV void rec_get(const RecoverParams& prm, int row, uint32_t idx, uint32_t out[8]) {
#pragma unroll
  for (int k = 0; k < 8; ++k) out[k] = prm.rec[(size_t)(row + k) * prm.n_pad + idx];
}

// Progress-balanced issue priority. Co-resident waves of a SIMD are otherwise arbitrated by
// age: the older wave finishes far ahead and the younger one then runs alone at a fraction
// of the issue rate (measured: per-wave lifetimes spread 1.8x). A wave lowers its priority
// as it advances (units: 1 per lift, 4 per ecmult), so lagging waves catch up and the SIMD
// keeps two waves busy to the end. p must be wave-uniform.
DEV void balance_prio(uint32_t done, uint32_t total) {
  const uint32_t q = __builtin_amdgcn_readfirstlane(total ? (4u * done) / total : 0u);
  switch (q) {
    case 0: __builtin_amdgcn_s_setprio(3); break;
    case 1: __builtin_amdgcn_s_setprio(2); break;
    case 2: __builtin_amdgcn_s_setprio(1); break;
    default: __builtin_amdgcn_s_setprio(0); break;
  }
}


// One signature per thread up to a full resident grid, then K = ceil(n / threads) per thread;
// more blocks than resident when that would exceed MAX_SLOTS signatures per thread.
inline int grid_for_lane_serial(uint32_t n, int max_blocks) {
  const uint32_t tiles = (n + WG - 1) / WG;
  uint32_t g = tiles < (uint32_t)max_blocks ? tiles : (uint32_t)max_blocks;
  const uint32_t min_g = (n + (uint32_t)WG * MAX_SLOTS - 1) / ((uint32_t)WG * MAX_SLOTS);
  return (int)(g > min_g ? g : min_g);
}


// ------------------------------------------------------------------ byte helpers
DEV void limbs_from_be32(uint32_t out[8], const uint8_t* b) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint8_t* q = b + 28 - 4 * i;
    out[i] = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | q[3];
  }
}
DEV void write_be32(uint8_t* dst, const uint32_t x[8]) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    uint32_t w = x[7 - i];
    dst[4 * i + 0] = (uint8_t)(w >> 24);
    dst[4 * i + 1] = (uint8_t)(w >> 16);
    dst[4 * i + 2] = (uint8_t)(w >> 8);
    dst[4 * i + 3] = (uint8_t)w;
  }
}
DEV uint64_t be_word(const uint32_t x[8], int k) {  // little-endian 64-bit word k of the BE encoding
  return (uint64_t)__builtin_bswap32(x[7 - 2 * k]) | ((uint64_t)__builtin_bswap32(x[6 - 2 * k]) << 32);
}

// Keccak-256(X || Y)[12:32] as 5 little-endian words; X, Y canonical 256-bit integers.
DEV void pub_address(uint32_t a[5], const uint32_t X[8], const uint32_t Y[8]) {
  uint64_t w[17];
#pragma unroll
  for (int k = 0; k < 17; ++k) w[k] = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    w[k] = be_word(X, k);
    w[4 + k] = be_word(Y, k);
  }
  uint64_t h[4];
  keccak256_1block<64>(w, h);
  a[0] = (uint32_t)(h[1] >> 32);
  a[1] = (uint32_t)h[2];
  a[2] = (uint32_t)(h[2] >> 32);
  a[3] = (uint32_t)h[3];
  a[4] = (uint32_t)(h[3] >> 32);
}

struct LatParse {
  sc R, Sv, Z;
  uint32_t xr[8];
  uint32_t meta, recid;
  bool ok;
};
// ------------------------------------------------------------------ record parse
// The signature's scalars, R's x and the pre-check status (main_impl.h:38-121) from the prep
// kernels' record rows, or (raw_sig set) from the caller's msg / sig bytes (the fused prep of
// prep_ecrecover_kernel, k_prep.hip). Wave-uniform in the latency kernels' row-form waves, per
// lane in the lane-serial ones (root helpers, the mid-size kernel).
DEV LatParse lat_parse(const RecoverParams& prm, uint32_t idx) {
  LatParse q;
  uint32_t rl[8], sl[8], zl[8];
  if (prm.raw_sig) {  // fused prep: prep_ecrecover_kernel's parse (k_prep.hip), same record
    const uint8_t* sg = prm.raw_sig + (size_t)idx * 65;
    limbs_from_be32(zl, prm.raw_msg + (size_t)idx * 32);
    limbs_from_be32(rl, sg);
    limbs_from_be32(sl, sg + 32);
    const uint32_t v = sg[64];
    q.meta = v >= 4 ? (ST_INVALID_RECOVERY_ID << 8) : v;  // checkSignature, secp256.go:171-179
  } else {
    rec_get(prm, 8, idx, rl);
    rec_get(prm, 16, idx, sl);
    rec_get(prm, 0, idx, zl);
    q.meta = prm.rec[(size_t)24 * prm.n_pad + idx];
  }
  q.recid = q.meta & 3u;
  q.ok = ((q.meta >> 8) & 0xffu) == ST_OK;
  bool ovr, ovs, ovz;
  q.R = sc_from_limbs(rl, ovr);
  q.Sv = sc_from_limbs(sl, ovs);
  q.Z = sc_from_limbs(zl, ovz);  // msg mod n (main_impl.h:183)
  q.ok = q.ok && !ovr && !ovs && !sc_is_zero(q.R) && !sc_is_zero(q.Sv);
#pragma unroll
  for (int i = 0; i < 8; ++i) q.xr[i] = q.R.v[i];
  if (q.recid & 2u) {  // x = r + n, only when r < p - n (main_impl.h:101-109)
    q.ok = q.ok && !u256_ge(q.R.v, P_MINUS_N);
    uint64_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      c += (uint64_t)q.xr[i] + SC_N[i];
      q.xr[i] = (uint32_t)c;
      c >>= 32;
    }
  }
  return q;
}

}  // namespace eges
