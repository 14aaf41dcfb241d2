#include <type_traits>

#include "core.cuh"
#include "modinv_row.cuh"

namespace eges {

// ------------------------------------------------------------------ recover kernel
// Lane-serial layout: the grid has GT = gridDim.x * WG threads and thread g owns the
// signatures idx = k * GT + g, k < K_g (K_g <= MAX_SLOTS). Each thread runs Montgomery's
// batch-inversion trick over its own K_g signatures, so the two exponentiations (r^-1 mod n and
// the final Z^-1 mod p) cost 1/K_g each per signature and run on all 64 lanes of every wave —
// no workgroup barrier, no idle waves. Per-signature state between the phases lives in the
// slot rows that follow the record rows (launch.h).
//
// Phase marks (diagnostic build only): 0 parse + sqrt, 1 r^-1 + u1/u2, 2 GLV + digits,
// 3 R table, 4 Strauss loop, 5 Z^-1, 6 affine + Keccak + stores.
//
template <class ST>
DEV void recover_body(const RecoverParams& prm, uint64_t* stamps) {
  __shared__ CoreLds L;
  ST st_;
  ST* st = &st_;
  uint4* const slot = recover_slots(prm.rec, prm.n_pad);
  const uint32_t np = prm.n_pad;
  const uint32_t GT = gridDim.x * WG;
  const uint32_t g = blockIdx.x * WG + threadIdx.x;
  const uint32_t K = g < prm.n ? (prm.n - g + GT - 1) / GT : 0;  // my signatures
  uint32_t okm = 0;
  const uint32_t units = 5u * K;
  // --- phase A: parse, lift R, prefix products of r
  sc pre = sc_one();
#pragma unroll 1
  for (uint32_t k = 0; k < K; ++k) {
    balance_prio(k, units);
    const uint32_t idx = k * GT + g;
    uint32_t rl[8];
    rec_get(prm, 8, idx, rl);
    const uint32_t meta = prm.rec[(size_t)24 * np + idx];
    const uint32_t recid = meta & 3u;
    bool ok = ((meta >> 8) & 0xffu) == ST_OK;
    // parse_compact: r, s >= n => failure (recovery/main_impl.h:38-58)
    bool ovr, ovs;
    sc R = sc_from_limbs(rl, ovr);
    {
      uint32_t sl[8];
      rec_get(prm, 16, idx, sl);
      const sc S = sc_from_limbs(sl, ovs);
      ok = ok && !ovr && !ovs && !sc_is_zero(R) && !sc_is_zero(S);
    }
    // x = r (+ n)  (main_impl.h:101-109)
    uint32_t xr[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) xr[i] = R.v[i];
    if (recid & 2u) {
      ok = ok && !u256_ge(R.v, P_MINUS_N);
      uint64_t c = 0;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        c += (uint64_t)xr[i] + SC_N[i];
        xr[i] = (uint32_t)c;
        c >>= 32;
      }
    }
    ge Rp;
    ok = ge_set_xo(Rp, fe_from_u256(xr), (recid & 1u) != 0) && ok;
    // failed signatures carry the generator and r = 1 so every later step stays well-defined
    const ge G = gen_point();
    Rp.x = fe_select(ok, Rp.x, G.x);
    Rp.y = fe_select(ok, Rp.y, G.y);
    pre = sc_mul(pre, sc_select(ok, R, sc_one()));
    slot_put_pt(slot, np, 0, idx, Rp);
    slot_put_sc(slot, np, 5, idx, pre);
    okm |= (ok ? 1u : 0u) << k;
  }
  st->mark(0);
  // --- phase B: one scalar inversion per wave: the 64 threads' products batched again across
  // the lanes, inverted once by the row-form safegcd
  sc rinv_acc = sc_inv_wave(pre);
  st->mark(1);
  // --- phase C: k = K-1 .. 0: r^-1, u1 = -z/r, u2 = s/r, Q = u2 R + u1 G, prefix products of Z
  fe zpre = fe_one();
#pragma unroll 1
  for (int k = (int)K - 1; k >= 0; --k) {
    balance_prio(K + 4u * (K - 1u - (uint32_t)k), units);
    const uint32_t idx = (uint32_t)k * GT + g;
    bool ok = (okm >> k) & 1u;
    sc rinv, u1, u2;
    {
      uint32_t l[8];
      bool ov;
      rec_get(prm, 8, idx, l);
      const sc R = sc_select(ok, sc_from_limbs(l, ov), sc_one());
      rinv = k > 0 ? sc_mul(rinv_acc, slot_get_sc(slot, np, 5, idx - GT)) : rinv_acc;
      rinv_acc = sc_mul(rinv_acc, R);
      rec_get(prm, 0, idx, l);
      const sc Z = sc_from_limbs(l, ov);  // msg mod n (main_impl.h:183)
      rec_get(prm, 16, idx, l);
      const sc S = sc_from_limbs(l, ov);
      u1 = sc_neg(sc_mul(rinv, Z));
      u2 = sc_select(ok, sc_mul(rinv, S), sc_one());
    }
    st->mark(1);
    const ge Rp = slot_get_pt(slot, np, 0, idx);
    park_put<8>(prm.ws, 0, rinv_acc.v);
    park_put<FE_LIMBS>(prm.ws, 8, zpre.v);
    gej Q;
    bool qinf;
    ecmult_core(Q, qinf, Rp, u2, u1, prm.gtab, prm.ws, L, st, diag_of(prm));
    park_get<8>(prm.ws, 0, rinv_acc.v);
    park_get<FE_LIMBS>(prm.ws, 8, zpre.v);
    ok = ok && !qinf;  // main_impl.h:120
    okm = (okm & ~(1u << k)) | ((ok ? 1u : 0u) << k);
    Q.z = fe_select(ok, Q.z, fe_one());
    zpre = fe_mul(zpre, Q.z);
    ge xy;
    xy.x = Q.x;
    xy.y = Q.y;
    slot_put_pt(slot, np, 0, idx, xy);
    ge zz;
    zz.x = Q.z;
    zz.y = zpre;
    slot_put_pt(slot, np, 7, idx, zz);
  }
  // --- phase D: one field inversion per wave, as phase B
  fe zinv_acc = fe_inv_wave_z(zpre);
  st->mark(5);
  // --- phase E: k = 0 .. K-1 (reverse of phase C's product order): affine, address, stores
#pragma unroll 1
  for (uint32_t k = 0; k < K; ++k) {
    const uint32_t idx = k * GT + g;
    const bool ok = (okm >> k) & 1u;
    const ge zz = slot_get_pt(slot, np, 7, idx);
    const fe zi = k + 1 < K ? fe_mul(zinv_acc, slot_get_pt(slot, np, 7, idx + GT).y) : zinv_acc;
    zinv_acc = fe_mul(zinv_acc, zz.x);
    const ge xy = slot_get_pt(slot, np, 0, idx);
    const fe zi2 = fe_sqr(zi);
    uint32_t X[8], Y[8];
    fe_to_u256(X, fe_normalize(fe_mul(xy.x, zi2)));
    fe_to_u256(Y, fe_normalize(fe_mul(xy.y, fe_mul(zi2, zi))));
    const uint32_t pre_st = (prm.rec[(size_t)24 * np + idx] >> 8) & 0xffu;
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
  st->mark(6);
  if constexpr (!std::is_same<ST, NoStamp>::value) {
    if ((threadIdx.x & 63) == 0) {
      const uint32_t w = blockIdx.x * (WG / 64) + (threadIdx.x >> 6);
#pragma unroll
      for (int i = 0; i < 8; ++i) stamps[(size_t)w * 8 + i] = st_.acc[i];
    }
  }
}

__global__ void __launch_bounds__(WG, 2) recover_kernel(RecoverParams prm) { recover_body<NoStamp>(prm, nullptr); }

#ifdef EGES_PHASE_STAMPS
__global__ void __launch_bounds__(WG, 2) recover_kernel_stamped(RecoverParams prm, uint64_t* stamps) {
  recover_body<Stamper>(prm, stamps);
}
#endif

// ------------------------------------------------------------------ launcher
hipError_t launch_recover(const RecoverParams& p, int max_blocks, int ws_blocks, hipStream_t st) {
  if (p.n == 0) return hipSuccess;
  const int grid = grid_for_lane_serial(p.n, max_blocks);
  if (grid > ws_blocks) return hipErrorInvalidValue;  // the kernel indexes ws by blockIdx.x
  hipLaunchKernelGGL(recover_kernel, dim3(grid), dim3(WG), 0, st, p);
  return hipGetLastError();
}

#ifdef EGES_PHASE_STAMPS
hipError_t launch_recover_stamped(const RecoverParams& p, int max_blocks, int ws_blocks, hipStream_t st, uint64_t* stamps) {
  if (p.n == 0) return hipSuccess;
  const int grid = grid_for_lane_serial(p.n, max_blocks);
  if (grid > ws_blocks) return hipErrorInvalidValue;
  hipLaunchKernelGGL(recover_kernel_stamped, dim3(grid), dim3(WG), 0, st, p, stamps);
  return hipGetLastError();
}
#endif

int lane_serial_grid(uint32_t n, int max_blocks) { return grid_for_lane_serial(n, max_blocks); }

int occupancy_recover() {
  int b = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, recover_kernel, WG, 0) != hipSuccess || b < 1) b = 1;
  return b;
}

}  // namespace eges
