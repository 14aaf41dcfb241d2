#include "core.cuh"

namespace eges {

// ------------------------------------------------------------------ verify kernel
// crypto.VerifySignature: ext.h:58-75 -> secp256k1.c:228-247 (parse_compact), :150-163 and
// eckey_impl.h:17-34 (pubkey parse), :293-308 (low-s), ecdsa_impl.h:203-271 (sig_verify).
//
// Only 33-byte keys need the (p+1)/4 square root (a third of a signature's work). Each tile of
// WG signatures is first partitioned in LDS — compressed keys first — so at most one wave of
// the tile mixes the two key types and every other wave skips the root (wave-uniform branch).
__global__ void __launch_bounds__(WG, 2) verify_kernel(VerifyParams prm) {
  __shared__ CoreLds L;
  __shared__ uint32_t perm[WG];
  __shared__ uint32_t wcnt[NWAVES];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint32_t ntiles = (prm.n + WG - 1) / WG;
#pragma unroll 1
  for (uint32_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    {
      const uint32_t i0 = tile * WG + tid;
      const bool comp = i0 < prm.n && prm.publen[i0] == 33;
      const uint64_t b = __ballot(comp);
      const uint64_t below = (1ull << lane) - 1ull;
      if (lane == 0) wcnt[wave] = (uint32_t)__popcll(b);
      __syncthreads();
      uint32_t before = 0, total = 0;
#pragma unroll
      for (int w = 0; w < NWAVES; ++w) {
        before += w < wave ? wcnt[w] : 0u;
        total += wcnt[w];
      }
      const uint32_t pos = comp ? before + (uint32_t)__popcll(b & below)
                                : total + ((uint32_t)wave * 64u - before) + (uint32_t)__popcll(~b & below);
      perm[pos] = i0;
      __syncthreads();
    }
    const uint32_t idx = perm[tid];
    const bool in = idx < prm.n;
    uint32_t zl[8], rl[8], sl[8], px[8], py[8];
    uint32_t plen = 0, pfx = 0;
    if (in) {
      limbs_from_be32(zl, prm.msg + (size_t)idx * 32);
      limbs_from_be32(rl, prm.sig + (size_t)idx * 64);
      limbs_from_be32(sl, prm.sig + (size_t)idx * 64 + 32);
      plen = prm.publen[idx];
      const uint8_t* pk = prm.pub + (size_t)idx * 65;
      pfx = pk[0];
      limbs_from_be32(px, pk + 1);
      if (plen == 65) limbs_from_be32(py, pk + 33);
      else
        for (int k = 0; k < 8; ++k) py[k] = 0;
    } else {
      for (int k = 0; k < 8; ++k) { zl[k] = rl[k] = sl[k] = px[k] = py[k] = 1u; }
    }
    bool ovr, ovs, ovz;
    sc R = sc_from_limbs(rl, ovr);
    sc S = sc_from_limbs(sl, ovs);
    sc Z = sc_from_limbs(zl, ovz);
    bool ok = in && !ovr && !ovs;
    // pubkey parse (eckey_impl.h:17-34): coordinates must be < p
    const bool x_ok = !u256_ge(px, FE_P), y_ok = !u256_ge(py, FE_P);
    const fe X = fe_from_u256(px), Y = fe_from_u256(py);
    const bool c33 = plen == 33 && (pfx == 2 || pfx == 3);
    const bool c65 = plen == 65 && (pfx == 4 || pfx == 6 || pfx == 7);
    ge P;
    bool pk_ok;
    {
      ge lifted;
      lifted.y = Y;
      bool lo = false;
      if (__any(c33)) lo = ge_set_xo(lifted, X, pfx == 3);
      ge full;
      full.x = X;
      full.y = Y;
      const bool hybrid_bad = (pfx == 6 || pfx == 7) && ((py[0] & 1u) != (pfx == 7 ? 1u : 0u));
      const bool on = ge_is_valid(full);
      pk_ok = (c33 && x_ok && lo) || (c65 && x_ok && y_ok && !hybrid_bad && on);
      P.x = X;
      P.y = fe_select(c33, lifted.y, Y);
    }
    ok = ok && pk_ok;
    // ecdsa_verify: high s rejected; sig_verify: r, s != 0
    ok = ok && !sc_is_high(S) && !sc_is_zero(R) && !sc_is_zero(S);
    const ge G = gen_point();
    P.x = fe_select(ok, P.x, G.x);
    P.y = fe_select(ok, P.y, G.y);
    S = sc_select(ok, S, sc_one());
    sc sinv = wg_batch_inv<ScalarOps>(S, ok, L.inv_scratch);
    sinv = sc_select(ok, sinv, sc_one());
    sc u1 = sc_mul(sinv, Z);
    sc u2 = sc_select(ok, sc_mul(sinv, R), sc_one());
    gej Q;
    bool qinf;
    ecmult_core(Q, qinf, P, u2, u1, prm.gtab, prm.ws, L);
    ok = ok && !qinf;
    // x(Q) mod n == r  <=>  r*Z^2 == X  or  (r < p - n and (r + n)*Z^2 == X)
    const fe xr = fe_from_u256(R.v);
    const fe z2 = fe_sqr(Q.z);
    bool eq = fe_equal(Q.x, fe_mul(xr, z2));
    const bool small = !u256_ge(R.v, P_MINUS_N);
    uint32_t rn[8];
    uint64_t c = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      c += (uint64_t)R.v[k] + SC_N[k];
      rn[k] = (uint32_t)c;
      c >>= 32;
    }
    const fe xrn = fe_from_u256(rn);
    eq = eq || (small && fe_equal(Q.x, fe_mul(xrn, z2)));
    if (in) prm.ok[idx] = (ok && eq) ? 1 : 0;
  }
}

// ------------------------------------------------------------------ launcher
static int grid_for(uint32_t n, int max_blocks) {
  const uint32_t tiles = (n + WG - 1) / WG;
  return (int)(tiles < (uint32_t)max_blocks ? tiles : (uint32_t)max_blocks);
}

hipError_t launch_verify(const VerifyParams& p, int max_blocks, hipStream_t st) {
  if (p.n == 0) return hipSuccess;
  hipLaunchKernelGGL(verify_kernel, dim3(grid_for(p.n, max_blocks)), dim3(WG), 0, st, p);
  return hipGetLastError();
}

int occupancy_verify() {
  int b = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, verify_kernel, WG, 0) != hipSuccess || b < 1) b = 1;
  return b;
}

}  // namespace eges
