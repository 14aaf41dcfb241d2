#pragma once
// Variable-time safegcd for the latency kernel (one signature per wave): the divsteps run on the
// scalar ALU (wave-uniform data), and the 2x2 transition-matrix update of the four 270-bit
// states f, g, d, e runs limb-parallel over a 16-lane row (lane L = signed radix-2^30 limb L,
// lanes 9..15 zero), so a batch costs a few dependent VALU steps instead of a 9-limb serial
// carry chain per state. Same values as modinv.cuh's constant-time modinv256 (Bernstein-Yang
// divsteps, variable-time here; update_de_30's md / me correction by M^-1 mod 2^30, after upstream libsecp256k1's
// modinv32, MIT).
//
// Limbs are kept "almost normalised" instead of exact: after each update, two parallel carry
// rounds (DPP row_shl / row_shr by one lane) leave limbs 0..7 in [-4, 2^30 + 4] and the top
// limb signed and small, so every product of the next update (|u|, |v| <= 2^30) fits its 64-bit
// lane. The low 30 bits of limb 0 are the value's low 30 bits, which is all the divsteps read.
// Two consequences of the redundancy, both handled exactly:
//   - g == 0 is detected as "all limbs zero"; a zero held in another form runs on to the cap
//     (26 batches >= 741 divsteps, the bound for 256-bit inputs), where further batches leave
//     the value unchanged;
//   - the sign terms of md / me read the top limb, which can disagree with the value's sign
//     near zero; d, e then stay within a few M of the usual (-2M, M), and the final reduction
//     on the scalar ALU brings d into [0, M) by exact comparison.
#include "fr.cuh"
#include "modinv.cuh"
#include "sc.cuh"

namespace eges {

// t / 2^30 (exact: lane 0's low 30 bits are zero) as almost-normalised limbs (see above)
DEV int32_t row_shift30(int64_t t) {
  const uint32_t L = row_lane();
  const int64_t h = t >> 30;                                // |h| <= 2^32
  const uint32_t ln = shl<1>((uint32_t)t & (uint32_t)M30);  // limb L+1's low 30 bits
  const int64_t r = h + (int64_t)ln;                        // weight 2^(30 L) of t / 2^30
  const int32_t h2 = (int32_t)(r >> 30);                    // in [-4, 5]
  const int32_t hp = (int32_t)shr<1>((uint32_t)h2);         // limb L-1's carry (0 into lane 0)
  const int32_t keep = L == 8 ? (int32_t)r : (int32_t)((uint32_t)r & (uint32_t)M30);
  return L <= 8 ? keep + hp : 0;
}

// canonical signed radix-2^30 (limbs 0..7 in [0, 2^30), limb 8 signed); wave-uniform
DEV void s30_carry(s30& a) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    a.v[i + 1] += a.v[i] >> 30;
    a.v[i] &= M30;
  }
}
// a >= b for canonical values
DEV bool s30_ge(const s30& a, const s30& b) {
#pragma unroll
  for (int i = 8; i >= 0; --i)
    if (a.v[i] != b.v[i]) return a.v[i] > b.v[i];
  return true;
}

// Variable-time divsteps (the "divsteps_n_matrix_var" form of the safegcd paper and of upstream
// libsecp256k1's modinv32_var, MIT; restated here) for wave-uniform f, g, 30 per batch: runs of
// zero bits of g are shifted out at once (count trailing zeros), and when g is odd up to
// min(eta + 1, remaining, 6) low bits of g are cancelled in one step by adding w f,
// w = -g f^-1 mod 2^k. eta = -delta, starting at -1 (delta = 1). Only for data that is uniform
// across a wave: the loops are data-dependent branches. The compiled C loop (round 3) and the
// lane-serial form it was restated from are in profiles/r06/removed_ab_branches_r06.diff.
//
// As scalar-ALU assembly (one wave alone issues ~1 instruction per 6-8
// cycles, tools/ubench_lat.hip, so the loop is priced by its instruction count):
//  - a swap happens in ~97 % of the iterations (the eta rule), so the loop is written twice with
//    the registers' roles exchanged (copy A: f = A, g = B, (u, v) = (uA, vA), (q, r) = (uB, vB);
//    copy B the other way round): a swap is three negations and a fall-through into the other
//    copy's tail, instead of six moves;
//  - the bits of g cancelled per iteration are capped at 6 (libsecp256k1's formula
//    w = f g (f^2 - 2) mod 2^6, f^-1 by one Newton step from f^-1 = f mod 8) instead of a 12-bit
//    inverse recomputed at every swap: a capped iteration is simply continued by the next one, so
//    the sequence of divsteps, and the (u, v, q, r) after 30 of them, are unchanged (the same
//    argument as libsecp256k1 modinv32_impl.h's variable-time divsteps);
//  - the remaining count i is kept as the sentinel mask sm = -1 << i (shifted arithmetically with
//    g), which gives ctz's sentinel, the end test (sm == -1) and the limit mask (~sm) directly.
// ~30 instructions per iteration (swap path) against ~41 for the compiled C version.
DEV int32_t divsteps_30_var_asm(int32_t eta, uint32_t f0, uint32_t g0, trans2x2& t) {
  uint32_t A = f0, B = g0, uA = 1, vA = 0, uB = 0, vB = 1, sm = 0xC0000000u;  // -1 << 30
  uint32_t tmp, z, m, w;
  asm volatile(
      "LA_head_%=:\n"
      "  s_or_b32 %[tmp], %[B], %[sm]\n"
      "  s_ff1_i32_b32 %[z], %[tmp]\n"
      "  s_lshr_b32 %[B], %[B], %[z]\n"
      "  s_lshl_b32 %[uA], %[uA], %[z]\n"
      "  s_lshl_b32 %[vA], %[vA], %[z]\n"
      "  s_sub_i32 %[eta], %[eta], %[z]\n"
      "  s_ashr_i32 %[sm], %[sm], %[z]\n"
      "  s_cmp_eq_u32 %[sm], -1\n"
      "  s_cbranch_scc1 LA_done_%=\n"
      "  s_cmp_lt_i32 %[eta], 0\n"
      "  s_cbranch_scc0 LA_tail_%=\n"
      // swap: (f, g) = (g, -f), (u, v, q, r) = (q, r, -u, -v), eta = -eta: copy B's roles
      "  s_sub_i32 %[eta], 0, %[eta]\n"
      "  s_sub_i32 %[A], 0, %[A]\n"
      "  s_sub_i32 %[uA], 0, %[uA]\n"
      "  s_sub_i32 %[vA], 0, %[vA]\n"
      "LB_tail_%=:\n"  // f = B, g = A, f-row (uB, vB), g-row (uA, vA); eta >= 0
      "  s_add_i32 %[tmp], %[eta], 1\n"
      "  s_min_u32 %[tmp], %[tmp], 6\n"
      "  s_bfm_b32 %[m], %[tmp], 0\n"
      "  s_andn2_b32 %[m], %[m], %[sm]\n"
      "  s_mul_i32 %[tmp], %[B], %[B]\n"
      "  s_add_i32 %[tmp], %[tmp], -2\n"
      "  s_mul_i32 %[tmp], %[tmp], %[B]\n"
      "  s_mul_i32 %[tmp], %[tmp], %[A]\n"
      "  s_and_b32 %[w], %[tmp], %[m]\n"
      "  s_mul_i32 %[tmp], %[B], %[w]\n"
      "  s_add_i32 %[A], %[A], %[tmp]\n"
      "  s_mul_i32 %[tmp], %[uB], %[w]\n"
      "  s_add_i32 %[uA], %[uA], %[tmp]\n"
      "  s_mul_i32 %[tmp], %[vB], %[w]\n"
      "  s_add_i32 %[vA], %[vA], %[tmp]\n"
      "LB_head_%=:\n"
      "  s_or_b32 %[tmp], %[A], %[sm]\n"
      "  s_ff1_i32_b32 %[z], %[tmp]\n"
      "  s_lshr_b32 %[A], %[A], %[z]\n"
      "  s_lshl_b32 %[uB], %[uB], %[z]\n"
      "  s_lshl_b32 %[vB], %[vB], %[z]\n"
      "  s_sub_i32 %[eta], %[eta], %[z]\n"
      "  s_ashr_i32 %[sm], %[sm], %[z]\n"
      "  s_cmp_eq_u32 %[sm], -1\n"
      "  s_cbranch_scc1 LB_done_%=\n"
      "  s_cmp_lt_i32 %[eta], 0\n"
      "  s_cbranch_scc0 LB_tail_%=\n"
      "  s_sub_i32 %[eta], 0, %[eta]\n"
      "  s_sub_i32 %[B], 0, %[B]\n"
      "  s_sub_i32 %[uB], 0, %[uB]\n"
      "  s_sub_i32 %[vB], 0, %[vB]\n"
      "LA_tail_%=:\n"  // f = A, g = B, f-row (uA, vA), g-row (uB, vB); eta >= 0
      "  s_add_i32 %[tmp], %[eta], 1\n"
      "  s_min_u32 %[tmp], %[tmp], 6\n"
      "  s_bfm_b32 %[m], %[tmp], 0\n"
      "  s_andn2_b32 %[m], %[m], %[sm]\n"
      "  s_mul_i32 %[tmp], %[A], %[A]\n"
      "  s_add_i32 %[tmp], %[tmp], -2\n"
      "  s_mul_i32 %[tmp], %[tmp], %[A]\n"
      "  s_mul_i32 %[tmp], %[tmp], %[B]\n"
      "  s_and_b32 %[w], %[tmp], %[m]\n"
      "  s_mul_i32 %[tmp], %[A], %[w]\n"
      "  s_add_i32 %[B], %[B], %[tmp]\n"
      "  s_mul_i32 %[tmp], %[uA], %[w]\n"
      "  s_add_i32 %[uB], %[uB], %[tmp]\n"
      "  s_mul_i32 %[tmp], %[vA], %[w]\n"
      "  s_add_i32 %[vB], %[vB], %[tmp]\n"
      "  s_branch LA_head_%=\n"
      "LB_done_%=:\n"  // copy B's roles back to (u, v) = (uA, vA), (q, r) = (uB, vB)
      "  s_mov_b32 %[tmp], %[uA]\n"
      "  s_mov_b32 %[uA], %[uB]\n"
      "  s_mov_b32 %[uB], %[tmp]\n"
      "  s_mov_b32 %[tmp], %[vA]\n"
      "  s_mov_b32 %[vA], %[vB]\n"
      "  s_mov_b32 %[vB], %[tmp]\n"
      "LA_done_%=:\n"
      : [A] "+s"(A), [B] "+s"(B), [uA] "+s"(uA), [vA] "+s"(vA), [uB] "+s"(uB), [vB] "+s"(vB), [sm] "+s"(sm),
        [eta] "+s"(eta), [tmp] "=&s"(tmp), [z] "=&s"(z), [m] "=&s"(m), [w] "=&s"(w)
      :
      : "scc");
  t.u = (int32_t)uA;
  t.v = (int32_t)vA;
  t.q = (int32_t)uB;
  t.r = (int32_t)vB;
  return eta;
}

// x^-1 mod M for x in [0, M), x wave-uniform (0 maps to 0)
// prof (diagnostic builds only): accumulates [0] divsteps ticks, [1] state-update ticks
template <class Mod>
DEV void modinv256_row_var(uint32_t out[8], const uint32_t x[8], uint64_t* prof = nullptr) {
  const uint32_t L = row_lane();
  const s30 xs = s30_from_u256(x);
  int32_t f = 0, g = 0, m = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    f = L == (uint32_t)i ? Mod::m[i] : f;
    g = L == (uint32_t)i ? xs.v[i] : g;
  }
  m = f;
  int32_t d = 0, e = L == 0 ? 1 : 0;
  int32_t eta = -1;
#pragma unroll 1
  for (int it = 0; it < 26; ++it) {
    trans2x2 t;
    const uint64_t p0 = prof ? __builtin_amdgcn_s_memtime() : 0;
    eta = divsteps_30_var_asm(eta, (uint32_t)__builtin_amdgcn_readlane(f, 0), (uint32_t)__builtin_amdgcn_readlane(g, 0), t);
    const uint64_t p1 = prof ? __builtin_amdgcn_s_memtime() : 0;
    // update_de_30's correction, from lane 0's limbs and the top limbs' signs
    const int32_t d0 = __builtin_amdgcn_readlane(d, 0), e0 = __builtin_amdgcn_readlane(e, 0);
    const int32_t sd = __builtin_amdgcn_readlane(d, 8) >> 31, se = __builtin_amdgcn_readlane(e, 8) >> 31;
    int32_t md = (t.u & sd) + (t.v & se);
    int32_t me = (t.q & sd) + (t.r & se);
    const int64_t cd0 = (int64_t)t.u * d0 + (int64_t)t.v * e0;
    const int64_t ce0 = (int64_t)t.q * d0 + (int64_t)t.r * e0;
    md -= (int32_t)((Mod::minv * (uint32_t)cd0 + (uint32_t)md) & (uint32_t)M30);
    me -= (int32_t)((Mod::minv * (uint32_t)ce0 + (uint32_t)me) & (uint32_t)M30);
    // the four states, limb-parallel
    const int64_t cf = (int64_t)t.u * f + (int64_t)t.v * g;
    const int64_t cg = (int64_t)t.q * f + (int64_t)t.r * g;
    const int64_t cd = (int64_t)t.u * d + (int64_t)t.v * e + (int64_t)m * md;
    const int64_t ce = (int64_t)t.q * d + (int64_t)t.r * e + (int64_t)m * me;
    f = row_shift30(cf);
    g = row_shift30(cg);
    d = row_shift30(cd);
    e = row_shift30(ce);
    const bool done = !__any(g != 0);
    if (prof) {
      prof[0] += p1 - p0;
      prof[1] += __builtin_amdgcn_s_memtime() - p1;
    }
    if (done) break;
  }
  // exact values on the scalar ALU: f = +-1, d == +-x^-1 (mod M)
  s30 fv, dv, mv;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    fv.v[i] = __builtin_amdgcn_readlane(f, i);
    dv.v[i] = __builtin_amdgcn_readlane(d, i);
    mv.v[i] = Mod::m[i];
  }
  s30_carry(fv);
  s30_carry(dv);
#pragma unroll 1
  while (dv.v[8] < 0) {
#pragma unroll
    for (int i = 0; i < 9; ++i) dv.v[i] += mv.v[i];
    s30_carry(dv);
  }
#pragma unroll 1
  while (s30_ge(dv, mv)) {
#pragma unroll
    for (int i = 0; i < 9; ++i) dv.v[i] -= mv.v[i];
    s30_carry(dv);
  }
  if (fv.v[8] < 0) {  // f == -1: negate (M - d, or 0)
    bool z = true;
#pragma unroll
    for (int i = 0; i < 9; ++i) z = z && dv.v[i] == 0;
    if (!z) {
#pragma unroll
      for (int i = 0; i < 9; ++i) dv.v[i] = mv.v[i] - dv.v[i];
      s30_carry(dv);
    }
  }
  s30_to_u256(out, dv);
}

// r^-1 / s^-1 mod n in the latency kernels (wave-uniform scalar in and out)
DEV sc sc_inv_row_var(const sc& a) {
  sc r;
  modinv256_row_var<ModN>(r.v, a.v);
  return r;
}

// Every lane's z^-1 (all 64 lanes active, every z nonzero mod p) by Montgomery's trick across the
// wave: inclusive prefix and suffix products by log-depth scans (cross-lane shuffles, 12 products),
// ONE inversion of the wave's product with the row-form variable-time safegcd above (the product
// is wave-uniform), then z_i^-1 = prod^-1 * prefix_(i-1) * suffix_(i+1). For the lane-serial
// kernels' final Z^-1 where one wave holds 64 signatures and its inversion is on the critical path
// (the mid-size kernel): ~15k VALU instructions of constant-time safegcd per lane become one
// variable-time inversion plus 14 products.
DEV fe fe_inv_wave(const fe& z) {
  const int lane = (int)lane_id();
  fe P = z;
#pragma unroll 1
  for (int d = 1; d < 64; d <<= 1) {
    const fe y = shfl_up_t(P, d);
    const fe m = fe_mul(P, y);
    P = fe_select(lane >= d, m, P);
  }
  fe Q = z;
#pragma unroll 1
  for (int d = 1; d < 64; d <<= 1) {
    const fe y = shfl_down_t(Q, d);
    const fe m = fe_mul(Q, y);
    Q = fe_select(lane + d < 64, m, Q);
  }
  const fe pex = fe_select(lane == 0, fe_one(), shfl_up_t(P, 1));
  const fe sex = fe_select(lane == 63, fe_one(), shfl_down_t(Q, 1));
  fe tot;
#pragma unroll
  for (int i = 0; i < FE_LIMBS; ++i) tot.v[i] = (uint32_t)__builtin_amdgcn_readlane((int)P.v[i], 63);
  uint32_t x[8], y[8];
  fe_to_u256(x, fe_normalize(tot));
  modinv256_row_var<ModP>(y, x);
  return fe_mul(fe_from_u256(y), fe_mul(pex, sex));
}

// The same for scalars mod n (the lane-serial kernels' batched r^-1 / s^-1): every lane's a^-1,
// every a nonzero mod n, one row-form inversion for the wave.
DEV sc sc_inv_wave(const sc& a) {
  const int lane = (int)lane_id();
  sc P = a;
#pragma unroll 1
  for (int d = 1; d < 64; d <<= 1) {
    const sc y = shfl_up_t(P, d);
    const sc m = sc_mul(P, y);
    P = sc_select(lane >= d, m, P);
  }
  sc Q = a;
#pragma unroll 1
  for (int d = 1; d < 64; d <<= 1) {
    const sc y = shfl_down_t(Q, d);
    const sc m = sc_mul(Q, y);
    Q = sc_select(lane + d < 64, m, Q);
  }
  const sc pex = sc_select(lane == 0, sc_one(), shfl_up_t(P, 1));
  const sc sex = sc_select(lane == 63, sc_one(), shfl_down_t(Q, 1));
  sc tot;
#pragma unroll
  for (int i = 0; i < 8; ++i) tot.v[i] = (uint32_t)__builtin_amdgcn_readlane((int)P.v[i], 63);
  sc inv;
  modinv256_row_var<ModN>(inv.v, tot.v);
  return sc_mul(inv, sc_mul(pex, sex));
}
// fe_inv_wave for values that may be zero (the lane-serial kernel's Z products): a zero lane gets
// 0 (as fe_inv(0)) without zeroing the rest of the wave's batch
DEV fe fe_inv_wave_z(const fe& z) {
  const bool zero = fe_is_zero(z);
  const fe r = fe_inv_wave(fe_select(zero, fe_one(), z));
  return fe_select(zero, fe_zero(), r);
}

// Z^-1 in the latency kernel: value replicated over the rows in, same out (row form)
DEV fr fr_inv_var(fr a, uint64_t* prof = nullptr) {
  uint32_t x[8], y[8];
  fe_to_u256(x, fe_normalize(fr_to_fe(a)));
  modinv256_row_var<ModP>(y, x, prof);
  return fe_to_fr(fe_from_u256(y));
}

}  // namespace eges
