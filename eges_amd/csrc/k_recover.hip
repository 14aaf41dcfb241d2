#include "core.cuh"

namespace eges {

// ------------------------------------------------------------------ recover kernel
__global__ void __launch_bounds__(WG, 2) recover_kernel(RecoverParams prm) {
  __shared__ CoreLds L;
  const int tid = threadIdx.x;
  const uint32_t ntiles = (prm.n + WG - 1) / WG;
#pragma unroll 1
  for (uint32_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const uint32_t idx = tile * WG + tid;
    const bool in = idx < prm.n;
    uint32_t zl[8], rl[8], sl[8], meta = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      zl[k] = in ? prm.rec[(size_t)k * prm.n_pad + idx] : 1u;
      rl[k] = in ? prm.rec[(size_t)(8 + k) * prm.n_pad + idx] : 1u;
      sl[k] = in ? prm.rec[(size_t)(16 + k) * prm.n_pad + idx] : 1u;
    }
    meta = in ? prm.rec[(size_t)24 * prm.n_pad + idx] : (ST_RECOVER_FAILED << 8);
    const uint32_t pre = (meta >> 8) & 0xffu;
    const uint32_t recid = meta & 3u;
    bool ok = in && pre == ST_OK;
    // parse_compact: r, s >= n => failure; secp256k1_ecdsa_recover: msg reduced mod n
    bool ovr, ovs, ovz;
    sc R = sc_from_limbs(rl, ovr);
    sc S = sc_from_limbs(sl, ovs);
    sc Z = sc_from_limbs(zl, ovz);
    ok = ok && !ovr && !ovs && !sc_is_zero(R) && !sc_is_zero(S);
    // x = r (+ n)
    uint32_t xr[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) xr[k] = R.v[k];
    if (recid & 2u) {
      ok = ok && !u256_ge(R.v, P_MINUS_N);
      uint64_t c = 0;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        c += (uint64_t)xr[k] + SC_N[k];
        xr[k] = (uint32_t)c;
        c >>= 32;
      }
    }
    const fe x = fe_from_u256(xr);
    ge Rp;
    const bool lifted = ge_set_xo(Rp, x, (recid & 1u) != 0);
    ok = ok && lifted;
    // failed lanes run on a dummy point / scalars so the arithmetic stays well-defined
    const ge G = gen_point();
    Rp.x = fe_select(ok, Rp.x, G.x);
    Rp.y = fe_select(ok, Rp.y, G.y);
    R = sc_select(ok, R, sc_one());
    sc rinv = wg_batch_inv<ScalarOps>(R, ok, L.inv_scratch);
    rinv = sc_select(ok, rinv, sc_one());
    sc u1 = sc_neg(sc_mul(rinv, Z));
    sc u2 = sc_mul(rinv, S);
    u2 = sc_select(ok, u2, sc_one());
    gej Q;
    bool qinf;
    ecmult_core(Q, qinf, Rp, u2, u1, prm.gtab, prm.ws, L);
    ok = ok && !qinf;
    // affine: batch-invert Z
    fe zi = wg_batch_inv<FieldOps>(Q.z, ok, L.inv_scratch);
    fe zi2 = fe_sqr(zi);
    uint32_t X[8], Y[8];
    fe_to_u256(X, fe_normalize(fe_mul(Q.x, zi2)));
    fe_to_u256(Y, fe_normalize(fe_mul(Q.y, fe_mul(zi2, zi))));
    if (in) {
      const uint32_t st = pre != ST_OK ? pre : (ok ? ST_OK : ST_RECOVER_FAILED);
      prm.status[idx] = (uint8_t)st;
      if (prm.addr) {
        uint32_t a[5];
        pub_address(a, X, Y);
        uint32_t* dst = reinterpret_cast<uint32_t*>(prm.addr + (size_t)idx * 20);
#pragma unroll
        for (int k = 0; k < 5; ++k) dst[k] = ok ? a[k] : 0u;
      }
      if (prm.pub) {
        uint8_t* dst = prm.pub + (size_t)idx * 65;
        if (ok) {
          dst[0] = 4;
          write_be32(dst + 1, X);
          write_be32(dst + 33, Y);
        } else {
          for (int k = 0; k < 65; ++k) dst[k] = 0;
        }
      }
    }
  }
}

// ------------------------------------------------------------------ launcher
static int grid_for(uint32_t n, int max_blocks) {
  const uint32_t tiles = (n + WG - 1) / WG;
  return (int)(tiles < (uint32_t)max_blocks ? tiles : (uint32_t)max_blocks);
}

hipError_t launch_recover(const RecoverParams& p, int max_blocks, hipStream_t st) {
  if (p.n == 0) return hipSuccess;
  hipLaunchKernelGGL(recover_kernel, dim3(grid_for(p.n, max_blocks)), dim3(WG), 0, st, p);
  return hipGetLastError();
}

int occupancy_recover() {
  int b = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, recover_kernel, WG, 0) != hipSuccess || b < 1) b = 1;
  return b;
}

}  // namespace eges
