// Wire-format transactions -> sender-batch rows on the GPU (SURVEY.md §8(f) N1 + N4).
//
// One wave per transaction up to 8192 items (tx_rows_wave_kernel), one thread per transaction
// above (tx_rows_kernel). Input: the RLP encoding of one txdata (what rlp.DecodeBytes(raw, tx)
// consumes, core/types/transaction.go:157-165); item first + i lies at
// raw[offsets[first + i] - offsets[0], offsets[first + i + 1] - offsets[0]).
// The wave (thread)
//   1. decodes it with the reference decoder's acceptance rules for the 10-field Geec txdata
//      struct (transaction.go:59-76; rlp/decode.go: readKind :937-984 and readUint :986-1008,
//      Kind's bound checks :874-907, uint :707-737, Bool :742-756, decodeBigInt :254-269,
//      Bytes :668-688, decodeByteArray :390-425, makeOptionalPtrDecoder :464-490 (rlp:"nil"),
//      the struct decoder's too-few / too-many checks :418-435, DecodeBytes' trailing-bytes
//      check :119-129). Any error sets VF_DECODE_ERR: the item gets EGES_DECODE_FAILED.
//   2. builds the signing payload — FrontierSigner.Hash (transaction_signing.go:207-216) or, for
//      a protected V under an EIP155 signer, EIP155Signer.Hash (:155-165) with the signer's chain
//      id — and Keccak-256s it (rlpHash, block.go:134-139). Every field except `to` re-encodes to
//      its canonical input bytes (the decoder rejected non-canonical forms), so the payload is
//      a new list header + raw[nonce .. payload] + (chainId, 0, 0); a nil `to` received as 0xC0
//      re-encodes as 0x80.
//   3. writes the sighash, V/R/S (32-byte big-endian, EGES_VF_*_WIDE when > 256 bits) and flags:
//      exactly the rows prep_sender_kernel takes (k_prep.hip), so the recovery is unchanged.
#include "core.cuh"
#include "keccak_wave.cuh"
#include "rlp.cuh"

#include <cstdlib>

namespace eges {

// Lane-serial form: one thread per transaction (large batches).
__global__ void __launch_bounds__(256) tx_rows_kernel(const uint8_t* __restrict__ raw,
                                                      const uint64_t* __restrict__ offsets, uint64_t first,
                                                      uint32_t n, int signer, uint64_t chain_id,
                                                      uint8_t* __restrict__ sighash, uint8_t* __restrict__ rr,
                                                      uint8_t* __restrict__ sr, uint8_t* __restrict__ vr,
                                                      uint8_t* __restrict__ vflags) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t raw_base = offsets[0], a = offsets[first + i], e = offsets[first + i + 1];
  uint8_t* const hout = sighash + (size_t)i * 32;
  uint8_t* const rout = rr + (size_t)i * 32;
  uint8_t* const sout = sr + (size_t)i * 32;
  uint8_t* const vout = vr + (size_t)i * 32;
  RlpHead f[10]{};
  Payload m;
  const bool ok = e >= a && a >= raw_base && tx_parse(raw + (a - raw_base), e - a, signer, chain_id, f, m);
  if (!ok) {
    for (int k = 0; k < 32; ++k) hout[k] = rout[k] = sout[k] = vout[k] = 0;
    vflags[i] = VF_DECODE_ERR;
    return;
  }
  uint32_t fl = 0;
  fl |= rlp_to_be32(m.p, f[7], vout) ? 0u : 1u;  // EGES_VF_V_WIDE
  fl |= rlp_to_be32(m.p, f[8], rout) ? 0u : 2u;  // EGES_VF_R_WIDE
  fl |= rlp_to_be32(m.p, f[9], sout) ? 0u : 4u;  // EGES_VF_S_WIDE
  keccak256_payload(m, hout);
  vflags[i] = (uint8_t)fl;
}

// Wave form: one wave per transaction (blocks and small batches, where the lane-serial form is
// one thread's chain of dependent global byte loads and two serial Keccak-f). The wave stages
// the encoding into LDS with coalesced loads, every lane runs the (wave-uniform) decode out of
// LDS, the payload's rate words are gathered one per lane and the permutation runs across the
// wave (keccak_wave.cuh); lanes 0..31 write the V/R/S rows.
constexpr int TXW_WAVES = 4;      // waves per workgroup
constexpr int TXW_STAGE = 1024;   // staged bytes per wave; longer encodings decode from global memory
// Up to block-sized batches the wave form wins (C3 from wire bytes: 0.325 -> 0.261 ms/block);
// at 10k transfers the two tie, and beyond the lane-serial form does (100k: 1.91 vs 2.26 ms).

// Big-endian integer content -> byte `lane` of the 32-byte row (lanes 0..31).
DEV uint32_t rlp_be32_byte(const uint8_t* __restrict__ p, const RlpHead& h, uint32_t lane) {
  const uint64_t len = h.kind == RK_BYTE ? 1 : h.size;
  const int j = (int)lane - (32 - (int)len);
  const uint32_t b = p[(len <= 32 && j >= 0) ? h.off + j : h.start];  // in-bounds either way (rlp.cuh)
  return (len <= 32 && j >= 0) ? b : 0u;
}

__global__ void __launch_bounds__(64 * TXW_WAVES) tx_rows_wave_kernel(
    const uint8_t* __restrict__ raw, const uint64_t* __restrict__ offsets, uint64_t first, uint32_t n, int signer,
    uint64_t chain_id, uint8_t* __restrict__ sighash, uint8_t* __restrict__ rr, uint8_t* __restrict__ sr,
    uint8_t* __restrict__ vr, uint8_t* __restrict__ vflags) {
  __shared__ uint8_t stage[TXW_WAVES][TXW_STAGE];
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint32_t i = blockIdx.x * TXW_WAVES + w;  // wave-uniform
  if (i >= n) return;
  const uint64_t raw_base = offsets[0], a = offsets[first + i], e = offsets[first + i + 1];
  const bool span_ok = e >= a && a >= raw_base;
  const uint64_t len = span_ok ? e - a : 0;
  const uint8_t* src = raw + (span_ok ? a - raw_base : 0);
  if (len <= TXW_STAGE) {
    for (uint32_t j = lane; j < len; j += 64) stage[w][j] = src[j];
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    src = stage[w];
  }
  RlpHead f[10]{};
  Payload m;
  const bool ok = span_ok && tx_parse(src, len, signer, chain_id, f, m);
  uint8_t* const hout = sighash + (size_t)i * 32;
  if (!ok) {
    if (lane < 32) hout[lane] = rr[(size_t)i * 32 + lane] = sr[(size_t)i * 32 + lane] = vr[(size_t)i * 32 + lane] = 0;
    if (lane == 0) vflags[i] = VF_DECODE_ERR;
    return;
  }
  if (lane < 32) {
    vr[(size_t)i * 32 + lane] = (uint8_t)rlp_be32_byte(src, f[7], lane);
    rr[(size_t)i * 32 + lane] = (uint8_t)rlp_be32_byte(src, f[8], lane);
    sr[(size_t)i * 32 + lane] = (uint8_t)rlp_be32_byte(src, f[9], lane);
  }
  // Keccak-256 sponge, rate 136: lane w < 17 absorbs rate word w of each block
  const uint64_t M = m.length();
  const uint64_t nblk = M / 136 + 1;
  uint64_t st = 0;
#pragma unroll 1
  for (uint64_t b = 0; b < nblk; ++b) {
    if (lane < 17) {
      uint64_t x = 0;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const uint64_t j = b * 136 + 8 * lane + k;
        uint64_t byte = j < M ? m.at(j) : 0u;
        if (j == M) byte ^= 0x01u;
        if (b + 1 == nblk && 8 * lane + k == 135) byte ^= 0x80u;
        x |= byte << (8 * k);
      }
      st ^= x;
    }
    keccak_f1600_wave(st);
  }
  if (lane < 4) {
#pragma unroll
    for (int k = 0; k < 8; ++k) hout[8 * lane + k] = (uint8_t)(st >> (8 * k));
  }
  if (lane == 0) {
    uint32_t fl = 0;
    fl |= f[7].kind != RK_BYTE && f[7].size > 32 ? 1u : 0u;  // EGES_VF_V_WIDE
    fl |= f[8].kind != RK_BYTE && f[8].size > 32 ? 2u : 0u;  // EGES_VF_R_WIDE
    fl |= f[9].kind != RK_BYTE && f[9].size > 32 ? 4u : 0u;  // EGES_VF_S_WIDE
    vflags[i] = (uint8_t)fl;
  }
}

hipError_t launch_tx_rows(const uint8_t* raw, const uint64_t* offsets, uint64_t first, uint32_t n, int signer,
                          uint64_t chain_id, uint8_t* sighash, uint8_t* r, uint8_t* s, uint8_t* v, uint8_t* vflags,
                          hipStream_t st) {
  // KNOB_TXROWS_WAVE_MAX (default 8192, engine.hip) sets the cut (0: never the wave form)
  const uint32_t wave_max = (uint32_t)std::max<long long>(0, std::min<long long>(knob(KNOB_TXROWS_WAVE_MAX), 1u << 30));
  if (n <= wave_max)
    hipLaunchKernelGGL(tx_rows_wave_kernel, dim3((n + TXW_WAVES - 1) / TXW_WAVES), dim3(64 * TXW_WAVES), 0, st, raw,
                       offsets, first, n, signer, chain_id, sighash, r, s, v, vflags);
  else
    hipLaunchKernelGGL(tx_rows_kernel, dim3((n + 255) / 256), dim3(256), 0, st, raw, offsets, first, n, signer,
                       chain_id, sighash, r, s, v, vflags);
  return hipGetLastError();
}

}  // namespace eges
