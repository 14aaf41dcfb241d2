#include "core.cuh"
#include "modinv_row.cuh"

namespace eges {

// ------------------------------------------------------------------ verify kernels
// crypto.VerifySignature: ext.h:58-75 -> secp256k1.c:228-247 (parse_compact), :150-163 and
// eckey_impl.h:17-34 (pubkey parse), :293-308 (low-s), ecdsa_impl.h:203-271 (sig_verify).
//
// Same execution model as the recover kernel (k_recover.hip): thread g owns the items
// j = k * GT + g of a processing order, runs Montgomery's batch inversion of s over its own
// K items (one scalar inversion per thread, no workgroup barrier) and never needs a field
// inversion: x(Q) == r is checked projectively (r Z^2 == X).
//
// Only 33-byte keys need the (p+1)/4 square root, about a third of an item's work. The order
// kernel puts compressed keys first, so a wave's lanes hold the same key type at almost every
// step and the waves of uncompressed steps skip the root (wave-uniform branch).

// order: compressed keys from the front, the rest from the back (wave-aggregated atomics).
__global__ void __launch_bounds__(WG) verify_order_kernel(const uint8_t* publen, uint32_t n, uint32_t* order,
                                                          uint32_t* counts) {
  const uint32_t idx = blockIdx.x * WG + threadIdx.x;
  const int lane = threadIdx.x & 63;
  const bool in = idx < n;
  const bool comp = in && publen[idx] == 33;
  const uint64_t bc = __ballot(comp), bu = __ballot(in && !comp);
  const uint64_t below = (1ull << lane) - 1ull;
  uint32_t base_c = 0, base_u = 0;
  if (lane == 0) {
    if (bc) base_c = atomicAdd(&counts[0], (uint32_t)__popcll(bc));
    if (bu) base_u = atomicAdd(&counts[1], (uint32_t)__popcll(bu));
  }
  base_c = (uint32_t)__shfl((int)base_c, 0, 64);
  base_u = (uint32_t)__shfl((int)base_u, 0, 64);
  if (comp) order[base_c + (uint32_t)__popcll(bc & below)] = idx;
  else if (in) order[n - 1u - (base_u + (uint32_t)__popcll(bu & below))] = idx;
}

struct VerifyItem {
  sc R, S, Z;
  bool ok;  // parse and range checks passed
};

DEV VerifyItem verify_parse(const VerifyParams& prm, uint32_t idx) {
  VerifyItem it;
  uint32_t l[8];
  bool ovr, ovs, ovz;
  limbs_from_be32(l, prm.sig + (size_t)idx * 64);
  it.R = sc_from_limbs(l, ovr);
  limbs_from_be32(l, prm.sig + (size_t)idx * 64 + 32);
  it.S = sc_from_limbs(l, ovs);
  limbs_from_be32(l, prm.msg + (size_t)idx * 32);
  it.Z = sc_from_limbs(l, ovz);  // the message reduced mod n (ecdsa_impl.h:203-271)
  // parse_compact overflow => failure; ecdsa_verify rejects high s; sig_verify r, s != 0
  it.ok = !ovr && !ovs && !sc_is_high(it.S) && !sc_is_zero(it.R) && !sc_is_zero(it.S);
  return it;
}

__global__ void __launch_bounds__(WG, 2) verify_kernel(VerifyParams prm) {
  __shared__ CoreLds L;
  uint4* const slot = prm.slot;
  const uint32_t np = prm.n_pad;
  const uint32_t GT = gridDim.x * WG;
  const uint32_t g = blockIdx.x * WG + threadIdx.x;
  const uint32_t K = g < prm.n ? (prm.n - g + GT - 1) / GT : 0;
  const uint32_t units = 5u * K;
  uint32_t okm = 0;
  // --- phase A: parse, public key (lift 33-byte keys), prefix products of s
  sc pre = sc_one();
#pragma unroll 1
  for (uint32_t k = 0; k < K; ++k) {
    balance_prio(k, units);
    const uint32_t j = k * GT + g;
    const uint32_t idx = prm.order[j];
    const VerifyItem it = verify_parse(prm, idx);
    uint32_t px[8], py[8];
    const uint32_t plen = prm.publen[idx];
    const uint8_t* pk = prm.pub + (size_t)idx * 65;
    const uint32_t pfx = pk[0];
    limbs_from_be32(px, pk + 1);
    if (plen == 65) limbs_from_be32(py, pk + 33);
    else
      for (int q = 0; q < 8; ++q) py[q] = 0;
    // pubkey parse (eckey_impl.h:17-34): coordinates must be < p
    const bool x_ok = !u256_ge(px, FE_P), y_ok = !u256_ge(py, FE_P);
    const fe X = fe_from_u256(px), Y = fe_from_u256(py);
    const bool c33 = plen == 33 && (pfx == 2 || pfx == 3);
    const bool c65 = plen == 65 && (pfx == 4 || pfx == 6 || pfx == 7);
    ge lifted;
    lifted.y = Y;
    bool lo = false;
    if (__any(c33)) lo = ge_set_xo(lifted, X, pfx == 3);
    ge full;
    full.x = X;
    full.y = Y;
    const bool hybrid_bad = (pfx == 6 || pfx == 7) && ((py[0] & 1u) != (pfx == 7 ? 1u : 0u));
    const bool on = ge_is_valid(full);
    const bool pk_ok = (c33 && x_ok && lo) || (c65 && x_ok && y_ok && !hybrid_bad && on);
    const bool ok = it.ok && pk_ok;
    // failed items carry the generator and s = 1 so every later step stays well-defined
    const ge G = gen_point();
    ge P;
    P.x = fe_select(ok, X, G.x);
    P.y = fe_select(ok, fe_select(c33, lifted.y, Y), G.y);
    pre = sc_mul(pre, sc_select(ok, it.S, sc_one()));
    slot_put_pt(slot, np, 0, j, P);
    slot_put_sc(slot, np, 5, j, pre);
    okm |= (ok ? 1u : 0u) << k;
  }
  // --- phase B: one scalar inversion per wave (as k_recover.hip phase B)
  sc sinv_acc = sc_inv_wave(pre);
  // --- phase C: k = K-1 .. 0: s^-1, u1 = z/s, u2 = r/s, Q = u2 P + u1 G, x(Q) == r
#pragma unroll 1
  for (int k = (int)K - 1; k >= 0; --k) {
    balance_prio(K + 4u * (K - 1u - (uint32_t)k), units);
    const uint32_t j = (uint32_t)k * GT + g;
    const uint32_t idx = prm.order[j];
    bool ok = (okm >> k) & 1u;
    const VerifyItem it = verify_parse(prm, idx);
    const sc sinv = k > 0 ? sc_mul(sinv_acc, slot_get_sc(slot, np, 5, j - GT)) : sinv_acc;
    sinv_acc = sc_mul(sinv_acc, sc_select(ok, it.S, sc_one()));
    const sc u1 = sc_mul(sinv, it.Z);
    const sc u2 = sc_select(ok, sc_mul(sinv, it.R), sc_one());
    const ge P = slot_get_pt(slot, np, 0, j);
    park_put<8>(prm.ws, 0, sinv_acc.v);
    gej Q;
    bool qinf;
    ecmult_core<NoStamp>(Q, qinf, P, u2, u1, prm.gtab, prm.ws, L, nullptr, diag_of(prm));
    park_get<8>(prm.ws, 0, sinv_acc.v);
    ok = ok && !qinf;
    // x(Q) mod n == r  <=>  r*Z^2 == X  or  (r < p - n and (r + n)*Z^2 == X)  (ecdsa_impl.h:246-270)
    const fe xr = fe_from_u256(it.R.v);
    const fe z2 = fe_sqr(Q.z);
    bool eq = fe_equal(Q.x, fe_mul(xr, z2));
    const bool small = !u256_ge(it.R.v, P_MINUS_N);
    uint32_t rn[8];
    uint64_t c = 0;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      c += (uint64_t)it.R.v[q] + SC_N[q];
      rn[q] = (uint32_t)c;
      c >>= 32;
    }
    const fe xrn = fe_from_u256(rn);
    eq = eq || (small && fe_equal(Q.x, fe_mul(xrn, z2)));
    prm.ok[idx] = (ok && eq) ? 1 : 0;
  }
}

// ------------------------------------------------------------------ launcher
hipError_t launch_verify(const VerifyParams& p, int max_blocks, int ws_blocks, hipStream_t st) {
  if (p.n == 0) return hipSuccess;
  const int grid = grid_for_lane_serial(p.n, max_blocks);
  if (grid > ws_blocks) return hipErrorInvalidValue;  // the kernel indexes ws by blockIdx.x
  hipError_t e = hipMemsetAsync(p.counts, 0, 2 * sizeof(uint32_t), st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(verify_order_kernel, dim3((p.n + WG - 1) / WG), dim3(WG), 0, st, p.publen, p.n, p.order, p.counts);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(verify_kernel, dim3(grid), dim3(WG), 0, st, p);
  return hipGetLastError();
}

int occupancy_verify() {
  int b = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, verify_kernel, WG, 0) != hipSuccess || b < 1) b = 1;
  return b;
}

}  // namespace eges
