#pragma once
// Row-form field arithmetic mod p for the latency path (gfx950): one field element spread over
// a 16-lane DPP row, limb-parallel.
//
// The throughput kernels (fe.cuh) give every lane its own signature and a whole 9-limb element;
// one signature then costs one lane's serial instruction chain (~333k instructions, ~0.78 ms on
// a lightly loaded SIMD). For small batches (a 1000-transaction Geec block, single calls) the
// latency kernel (k_recover_lat.hip) gives every signature a whole wavefront instead: each
// field element lives in one VGPR of a 16-lane row (lane L = limb L of the radix-2^29 value,
// lanes 9..15 zero), and the four rows of the wave compute up to four independent field
// products of the same signature at once (quad steps, frg.cuh).
//
// Product a*b in a row: lane L accumulates column L = sum_i a_i b_(L-i) with a_i broadcast by
// DPP row_newbcast and b shifted by DPP row_shr (zero fill), one v_mad_u64_u32 per term, so
// every lane does 9 MADs instead of 81. Column 16 = a_8 b_8 is the row-uniform "tail". The
// reduction is three parallel carry rounds (DPP row_shr:1) around one fold of columns 9..17
// into 0..8 with 2^261 == 2^37 + 31264 (mod p) (DPP row_shl:8 / :9), and a last fold of the
// carry out of limb 8. (The lane-level model of this product and reduction that the bounds in
// the comments come from is tests/test_fr_model.py, checked there on the CPU against big
// integers at worst-case and random magnitudes and every fr_mul_sub preset.) Same values as libsecp256k1's field (field_10x26_impl.h:440,769); the
// representation is this engine's own.
//
// Magnitude (as fe.cuh): every limb <= m * 2^29 (limb 0 may carry up to 2^18 more). fr_mul /
// fr_sqr need m(a) * m(b) <= 6.5 and return m = 1; fr_sub<M>(a, b) needs m(b) < 2M and
// returns m(a) + 2M, at most 7. Lanes 9..15 are kept zero by every operation.
#include "fe.cuh"

namespace eges {

// ------------------------------------------------------------------ lanes and DPP
DEV uint32_t lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }
DEV uint32_t row_lane() { return lane_id() & 15u; }
DEV uint32_t row_id() { return lane_id() >> 4; }

// lane L of each row <- lane I of the same row
template <int I>
DEV uint32_t bcast(uint32_t x) {
  static_assert(I >= 0 && I < 16, "row_newbcast");
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x150 + I, 0xF, 0xF, true);
}
// lane L <- lane L - I of the same row, 0 for L < I
template <int I>
DEV uint32_t shr(uint32_t x) {
  static_assert(I >= 1 && I < 16, "row_shr");
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x110 + I, 0xF, 0xF, true);
}
// lane L <- lane L + I of the same row, 0 for L + I > 15
template <int I>
DEV uint32_t shl(uint32_t x) {
  static_assert(I >= 1 && I < 16, "row_shl");
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x100 + I, 0xF, 0xF, true);
}
// every row <- row R (LDS crossbar permute; no LDS memory used)
template <int R>
DEV uint32_t rep_row(uint32_t x) {
  const int addr = (int)((row_lane() + 16u * R) << 2);
  return (uint32_t)__builtin_amdgcn_ds_bpermute(addr, (int)x);
}

// ------------------------------------------------------------------ the element
struct fr {
  uint32_t v;  // limb row_lane() (0 for lanes 9..15)
};

// Row-lane constants, written as sums of independent selects so that they compile to
// v_cndmask (a nested ?: chain on the lane index becomes a branchy switch). 64p limbs per lane
// (fe.cuh fe_sub): 2^30 - 62528, 2^30 - 514, 2^30 - 2 (lanes 2..8), 0 (lanes 9..15).
DEV uint32_t lane_pick(uint32_t L, uint32_t l0, uint32_t v0, uint32_t l1, uint32_t v1) {
  return (L == l0 ? v0 : 0u) + (L == l1 ? v1 : 0u);
}
template <int M>
DEV uint32_t kconst() {
  const uint32_t L = row_lane();
  const uint32_t kk = 0x3FFFFFFEu * M;
  return (L <= 8 ? kk : 0u) + lane_pick(L, 0, 0x3FFF0BC0u * M - kk, 1, 0x3FFFFDFEu * M - kk);
}
DEV uint32_t cfold() {  // 2^261 == 31264 + 2^8 * 2^29 (mod p): factor per destination lane
  return lane_pick(row_lane(), 0, FOLD0, 1, 256u);
}
DEV uint32_t low9(uint32_t x) { return row_lane() <= 8 ? x : 0u; }

DEV fr fr_zero() { return fr{0u}; }
DEV fr fr_one() { return fr{row_lane() == 0 ? 1u : 0u}; }
DEV fr fr_small(uint32_t x) { return fr{row_lane() == 0 ? x : 0u}; }  // x < 2^29

DEV fr fr_add(fr a, fr b) { return fr{a.v + b.v}; }
template <int M>
DEV fr fr_sub(fr a, fr b) {
  static_assert(M >= 1 && M <= 3, "fr_sub: M in 1..3");
  return fr{a.v + kconst<M>() - b.v};
}
template <int M>
DEV fr fr_neg(fr a) { return fr_sub<M>(fr_zero(), a); }
DEV fr fr_mul_small(fr a, uint32_t k) { return fr{a.v * k}; }
DEV fr fr_select(bool c, fr a, fr b) { return fr{c ? a.v : b.v}; }

// The row-form carry chains have few dependent steps (round 5; a lone wave waits on each dependent
// instruction's latency). The round-4 code (two 64-bit carry rounds before the
// fold) is kept only as a patch, profiles/r06/removed_ab_branches_r06.diff.
// One parallel carry round: limbs < 2^32 -> magnitude 1 (limb 0 <= 2^29 + 2^18). (A four-step form
// that keeps limb 8's carry out of lane 9 instead of masking at the end measured no faster.)
DEV fr fr_normalize_weak(fr a) {
  const uint32_t c = a.v >> 29;
  const uint32_t e8 = bcast<8>(c);
  const uint32_t z = (a.v & M29) + cfold() * e8;
  return fr{low9(z + shr<1>(c))};
}

// ------------------------------------------------------------------ product
namespace frdetail {
template <int I>
DEV void mac(uint64_t& acc, uint32_t a, uint32_t b) {
  const uint32_t ai = bcast<I>(a);
  const uint32_t bi = shr<I>(b);
  acc = mad64(ai, bi, acc);
}
}  // namespace frdetail

// Shorter dependent chains (the same values as the round-4 code): carry rounds 1 and 2 replaced
// by one split of every column into 29 + 29 + 6 bits added into its own and the next two lanes
// (one level of independent shifts and masks, then one three-way add) before the fold and carry round 3; column 16's product takes its carries as the addend; the three MAD
// chains start from an inline 0 (no zeroed accumulators). Same-box A/Bs, profiles/r05/fr_*:
// C3 kernel 0.1683-0.1703 -> 0.1610-0.1622 ms, single recover p50 0.1124-0.1143 -> 0.108-0.110 ms.
DEV void fr_cols(uint64_t& col, uint32_t& a8, uint32_t& b8, fr a, fr b) {
  uint64_t c1, c2;
  col = mad64(bcast<0>(a.v), b.v, col);
  c1 = mad64(bcast<1>(a.v), shr<1>(b.v), 0);
  c2 = mad64(bcast<2>(a.v), shr<2>(b.v), 0);
  asm volatile("" : "+v"(c1), "+v"(c2));
  frdetail::mac<3>(col, a.v, b.v);
  frdetail::mac<4>(c1, a.v, b.v);
  frdetail::mac<5>(c2, a.v, b.v);
  frdetail::mac<6>(col, a.v, b.v);
  frdetail::mac<7>(c1, a.v, b.v);
  a8 = bcast<8>(a.v);
  b8 = bcast<8>(b.v);
  c2 = mad64(a8, shr<8>(b.v), c2);
  asm volatile("" : "+v"(c1), "+v"(c2));
  col += c1 + c2;
}
// columns (lane L = column L, < 2^63.9) + a_8 b_8 (column 16) -> reduced row element, magnitude 1
// (limbs < 2^29 + 2^26, limb 0 < 2^29)
DEV fr fr_reduce(uint64_t col, uint32_t a8, uint32_t b8) {
  const uint32_t L = row_lane();
  const uint32_t lo = (uint32_t)col, hi = (uint32_t)(col >> 32);
  const uint32_t p0 = lo & M29;
  const uint32_t p1 = __builtin_amdgcn_alignbit(hi, lo, 29) & M29;
  const uint32_t p2 = hi >> 26;  // col >> 58, < 2^6
  // n_L = p0_L + p1_(L-1) + p2_(L-2) < 2^30.01; column 16 = a8 b8 + p1_15 + p2_14, column 17 gets p2_15
  const uint32_t n = p0 + shr<1>(p1) + shr<2>(p2);
  const uint32_t s16 = p1 + shr<1>(p2);
  const uint64_t T = mad64(a8, b8, (uint64_t)bcast<15>(s16));  // < 2^60.8
  const uint32_t t16 = (uint32_t)T & M29, t17 = (uint32_t)(T >> 29) + bcast<15>(p2);  // t17 < 2^32
  // fold columns 9..17 into 0..8 as the round-4 reduction did (a fold with the tail's terms
  // summed first and no lane selects measured no better: the tail path then sets the pace)
  uint32_t X = shl<9>(n);
  X = L == 7 ? t16 : X;
  uint32_t Y = shl<8>(n);
  Y = L == 0 ? 0u : Y;
  Y = L == 8 ? t16 : Y;
  const uint32_t c17 = lane_pick(L, 0, FOLD0 * 256u, 1, 65536u) + (L == 8 ? FOLD0 : 0u);
  const uint64_t R = mad64(Y, opaque_u32(256u), mad64(X, FOLD0, mad64(c17, t17, (uint64_t)n)));  // < 2^55.01
  // carry round 3, limb 8's carry (< 2^18.01) folded into lanes 0 and 1. Lanes 9..15 hold the
  // folded columns' leftovers: masked out of r and of the carries that move up (no final mask)
  const uint32_t e = (uint32_t)(R >> 29);  // < 2^26.01
  const uint32_t r = (uint32_t)R & (L <= 8 ? M29 : 0u);
  const uint32_t e7 = L <= 7 ? e : 0u;  // (limb 8's carry goes to lanes 0 and 1 instead)
  const uint64_t z = mad64(bcast<8>(e), cfold(), (uint64_t)r);  // < 2^33.01
  const uint32_t zc = (uint32_t)(z >> 29);  // 0 outside lanes 0, 1
  return fr{((uint32_t)z & M29) + shr<1>(e7 + zc)};
}
DEV fr fr_mul_col(fr a, fr b, uint64_t col) {
  uint32_t a8, b8;
  fr_cols(col, a8, b8, a, b);
  return fr_reduce(col, a8, b8);
}
DEV fr fr_mul(fr a, fr b) { return fr_mul_col(a, b, 0); }
DEV fr fr_sqr(fr a) { return fr_mul(a, a); }
template <int M, int SH = 0>
DEV fr fr_mul_sub(fr a, fr b, fr c) {
  static_assert(M >= 1 && M <= 3 && SH >= 0 && SH <= 3, "fr_mul_sub");
  return fr_mul_col(a, b, (uint64_t)(kconst<M>() - c.v) << SH);
}
template <int M, int SH = 0>
DEV fr fr_sqr_sub(fr a, fr c) { return fr_mul_sub<M, SH>(a, a, c); }

// ------------------------------------------------------------------ conversions
// row form -> lane-serial form. Values outside a quad step are replicated over the four rows,
// so row 0's limbs are the value: v_readlane puts each in an SGPR, and everything computed from
// them (normalisation, the variable-time inversion, serialisation, Keccak) is wave-uniform and
// compiles to scalar-ALU code, which runs beside the row-form VALU work instead of as a
// latency-bound single-lane VALU chain.
DEV fe fr_to_fe(fr a) {
  fe r;
#pragma unroll
  for (int i = 0; i < FE_LIMBS; ++i) r.v[i] = __builtin_amdgcn_readlane(a.v, i);
  return r;
}
// per-row form of the same (each row its own value; the self-test runs one item per row)
DEV fe fr_to_fe_row(fr a) {
  fe r;
  r.v[0] = bcast<0>(a.v);
  r.v[1] = bcast<1>(a.v);
  r.v[2] = bcast<2>(a.v);
  r.v[3] = bcast<3>(a.v);
  r.v[4] = bcast<4>(a.v);
  r.v[5] = bcast<5>(a.v);
  r.v[6] = bcast<6>(a.v);
  r.v[7] = bcast<7>(a.v);
  r.v[8] = bcast<8>(a.v);
  return r;
}
// lane-serial form (row-uniform) -> row form
DEV fr fe_to_fr(const fe& x) {
  const uint32_t L = row_lane();
  uint32_t v = 0;
#pragma unroll
  for (int i = 0; i < FE_LIMBS; ++i) v = L == (uint32_t)i ? x.v[i] : v;
  return fr{v};
}
DEV fr fr_normalize(fr a) { return fe_to_fr(fe_normalize(fr_to_fe(a))); }
DEV bool fr_is_zero(fr a) { return fe_is_zero(fr_to_fe(a)); }
DEV bool fr_equal(fr a, fr b) { return fr_is_zero(fr_sub<1>(a, b)); }

// ------------------------------------------------------------------ quad steps
// The latency kernel gives each signature a whole wave; a value used by the formulas is held
// "replicated" (all four rows alike). A quad step computes up to four independent products of
// one formula level at once, row r taking operands a_r, b_r (v_cndmask on the row), and hands
// the four results back replicated with gfx950's v_permlane16_swap / v_permlane32_swap
// (three VALU instructions for all four rows, no LDS round trip).
DEV uint32_t rowsel(uint32_t x0, uint32_t x1, uint32_t x2, uint32_t x3) {
  const uint32_t r = row_id();
  uint32_t v = x0;
  v = r == 1 ? x1 : v;
  v = r == 2 ? x2 : v;
  v = r == 3 ? x3 : v;
  return v;
}
DEV fr rowsel(fr a0, fr a1, fr a2, fr a3) { return fr{rowsel(a0.v, a1.v, a2.v, a3.v)}; }

// p = (p0, p1, p2, p3) by row -> each row's value replicated over the wave
DEV void rep4(uint32_t p, uint32_t& r0, uint32_t& r1, uint32_t& r2, uint32_t& r3) {
  const auto a = __builtin_amdgcn_permlane16_swap(p, p, false, false);      // (p0 p0 p2 p2), (p1 p1 p3 p3)
  const auto b = __builtin_amdgcn_permlane32_swap(a[0], a[0], false, false);  // (p0 x4), (p2 x4)
  const auto c = __builtin_amdgcn_permlane32_swap(a[1], a[1], false, false);  // (p1 x4), (p3 x4)
  r0 = b[0];
  r2 = b[1];
  r1 = c[0];
  r3 = c[1];
}
DEV void rep4(fr p, fr& r0, fr& r1, fr& r2, fr& r3) { rep4(p.v, r0.v, r1.v, r2.v, r3.v); }
DEV void rep2(fr p, fr& r0, fr& r1) {  // rows (0, 1) -> replicated
  const auto a = __builtin_amdgcn_permlane16_swap(p.v, p.v, false, false);
  const auto b = __builtin_amdgcn_permlane32_swap(a[0], a[0], false, false);
  const auto c = __builtin_amdgcn_permlane32_swap(a[1], a[1], false, false);
  r0.v = b[0];
  r1.v = c[0];
}

// Independent products in one pass (row r: a_r * b_r), results replicated.
DEV void fr_mul4(fr& r0, fr& r1, fr& r2, fr& r3, fr a0, fr b0, fr a1, fr b1, fr a2, fr b2, fr a3, fr b3) {
  rep4(fr_mul(rowsel(a0, a1, a2, a3), rowsel(b0, b1, b2, b3)), r0, r1, r2, r3);
}
DEV void fr_mul3(fr& r0, fr& r1, fr& r2, fr a0, fr b0, fr a1, fr b1, fr a2, fr b2) {
  fr r3;
  rep4(fr_mul(rowsel(a0, a1, a2, a2), rowsel(b0, b1, b2, b2)), r0, r1, r2, r3);
}
DEV void fr_mul2(fr& r0, fr& r1, fr a0, fr b0, fr a1, fr b1) {
  rep2(fr_mul(rowsel(a0, a1, a0, a1), rowsel(b0, b1, b0, b1)), r0, r1);
}

}  // namespace eges
