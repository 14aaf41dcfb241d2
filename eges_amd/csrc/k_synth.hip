#include "core.cuh"

namespace eges {

// ------------------------------------------------------------------ synthetic signer
// Deterministic synthetic workload (NOT the measured path): signs msg_i with key_i.
DEV void keccak_tag_index(uint32_t out[8], const char* tag, int taglen, uint64_t idx) {
  uint64_t w[17];
#pragma unroll
  for (int k = 0; k < 17; ++k) w[k] = 0;
  uint8_t buf[24];
  for (int k = 0; k < 24; ++k) buf[k] = 0;
  for (int k = 0; k < taglen; ++k) buf[k] = (uint8_t)tag[k];
  for (int k = 0; k < 8; ++k) buf[taglen + k] = (uint8_t)(idx >> (8 * k));
  const int len = taglen + 8;
  for (int k = 0; k < len; ++k) w[k >> 3] |= (uint64_t)buf[k] << (8 * (k & 7));
  // pad at byte len (<= 18): handled by explicit xor
  w[len >> 3] ^= 0x01ull << (8 * (len & 7));
  uint64_t A[25];
#pragma unroll
  for (int k = 0; k < 25; ++k) A[k] = k < 17 ? w[k] : 0;
  A[16] ^= 0x80ull << 56;
  keccak_f1600(A);
  // digest bytes 0..31 big-endian value -> limbs
  uint8_t d[32];
  for (int k = 0; k < 32; ++k) d[k] = (uint8_t)(A[k >> 3] >> (8 * (k & 7)));
  limbs_from_be32(out, d);
}

__global__ void __launch_bounds__(WG, 2) synth_sign_kernel(SynthParams prm) {
  __shared__ CoreLds L;
  const int tid = threadIdx.x;
  const uint32_t ntiles = (prm.n + WG - 1) / WG;
#pragma unroll 1
  for (uint32_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const uint32_t li = tile * WG + tid;
    const bool in = li < prm.n;
    const uint64_t gi = prm.first + li;
    uint32_t kl[8], ml[8], nl[8];
    keccak_tag_index(kl, "eges-key", 8, gi);
    if (prm.msg_in && in) limbs_from_be32(ml, prm.msg_in + (size_t)li * 32);
    else keccak_tag_index(ml, "eges-msg", 8, gi);
    keccak_tag_index(nl, "eges-nonce", 10, gi);
    bool ov;
    sc d = sc_from_limbs(kl, ov);
    if (sc_is_zero(d)) d = sc_one();
    sc kn = sc_from_limbs(nl, ov);
    if (sc_is_zero(kn)) kn = sc_one();
    sc z = sc_from_limbs(ml, ov);
    // R = k*G and Pub = d*G via the same core (variable-base part unused: u_r = 0 -> digits 0)
    const ge G = gen_point();
    gej Rj, Pj;
    bool rinf, pinf;
    ecmult_core(Rj, rinf, G, sc_zero(), kn, prm.gtab, prm.ws, L);
    ecmult_core(Pj, pinf, G, sc_zero(), d, prm.gtab, prm.ws, L);
    fe rzi = wg_batch_inv<FieldOps>(Rj.z, true, L.inv_scratch);
    fe pzi = wg_batch_inv<FieldOps>(Pj.z, true, L.inv_scratch);
    fe rzi2 = fe_sqr(rzi), pzi2 = fe_sqr(pzi);
    uint32_t Rx[8], Ry[8], Px[8], Py[8];
    fe_to_u256(Rx, fe_normalize(fe_mul(Rj.x, rzi2)));
    fe_to_u256(Ry, fe_normalize(fe_mul(Rj.y, fe_mul(rzi2, rzi))));
    fe_to_u256(Px, fe_normalize(fe_mul(Pj.x, pzi2)));
    fe_to_u256(Py, fe_normalize(fe_mul(Pj.y, fe_mul(pzi2, pzi))));
    // r = Rx mod n, recid = odd(Ry) | (Rx >= n) << 1
    bool rov;
    sc r = sc_from_limbs(Rx, rov);
    uint32_t recid = (Ry[0] & 1u) | (rov ? 2u : 0u);
    // s = k^-1 (z + r d)
    sc kinv = wg_batch_inv<ScalarOps>(kn, true, L.inv_scratch);
    sc s = sc_mul(kinv, sc_add(z, sc_mul(r, d)));
    if (sc_is_high(s)) {
      s = sc_neg(s);
      recid ^= 1u;
    }
    if (in) {
      if (prm.msg) write_be32(prm.msg + (size_t)li * 32, ml);
      uint8_t* sg = prm.sig + (size_t)li * 65;
      write_be32(sg, r.v);
      write_be32(sg + 32, s.v);
      sg[64] = (uint8_t)recid;
      uint32_t a[5];
      pub_address(a, Px, Py);
      uint32_t* dst = reinterpret_cast<uint32_t*>(prm.addr + (size_t)li * 20);
#pragma unroll
      for (int k = 0; k < 5; ++k) dst[k] = a[k];
    }
  }
}

// ------------------------------------------------------------------ launcher
static int grid_for(uint32_t n, int max_blocks) {
  const uint32_t tiles = (n + WG - 1) / WG;
  return (int)(tiles < (uint32_t)max_blocks ? tiles : (uint32_t)max_blocks);
}

hipError_t launch_synth(const SynthParams& p, int max_blocks, hipStream_t st) {
  if (p.n == 0) return hipSuccess;
  hipLaunchKernelGGL(synth_sign_kernel, dim3(grid_for(p.n, max_blocks)), dim3(WG), 0, st, p);
  return hipGetLastError();
}

int occupancy_synth() {
  int b = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, synth_sign_kernel, WG, 0) != hipSuccess || b < 1) b = 1;
  return b;
}

}  // namespace eges
