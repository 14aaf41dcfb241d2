#pragma once
// types.Sender classification of one signature (transaction_signing.go:127-137,182-184,218-247,
// crypto.go:181-192, transaction.go:142-149, deriveChainId :250-260): items that fail before
// the C call get their Go error as status; the rest become ecrecover records with recid = v.
// Shared by prep_sender_kernel (k_prep.hip) and the fused wire-format mid-size kernel.
#include "core.cuh"

namespace eges {

DEV int bitlen_limbs(const uint32_t x[8]) {
  int bl = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i)
    if (x[i]) bl = 32 * i + (32 - __clz(x[i]));
  return bl;
}

// r, s, v: little-endian limbs of the 32-byte rows; f: the row's vflags (EGES_VF_*_WIDE bits,
// VF_DECODE_ERR). Returns meta = recid | status << 8 (the record row's word 24).
DEV uint32_t sender_meta(const uint32_t r[8], const uint32_t s[8], const uint32_t v[8], uint32_t f, int signer,
                         uint64_t chain_id) {
  const bool v_wide = f & 1u, r_wide = f & 2u, s_wide = f & 4u;
  // wire-format batches (k_txhash.hip): rlp.DecodeBytes failed, the tx never reaches Sender
  uint32_t status = (f & VF_DECODE_ERR) ? ST_DECODE_FAILED : ST_OK;
  bool homestead = signer != 0;
  // Vb: the V handed to recoverPlain
  uint32_t vb8[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) vb8[k] = v[k];
  bool vb_wide = v_wide;
  if (signer == 2 && status == ST_OK) {
    const int bl = v_wide ? 1000 : bitlen_limbs(v);
    const bool prot = bl <= 8 ? !(v[0] == 27u || v[0] == 28u) : true;
    if (prot) {
      bool match;
      if (bl <= 64) {
        const uint64_t vv = (uint64_t)v[0] | ((uint64_t)v[1] << 32);
        const uint64_t cid = (vv == 27 || vv == 28) ? 0 : (vv - 35) / 2;  // uint64 wrap as Go
        match = cid == chain_id;
      } else if (v_wide) {
        match = false;
      } else {
        // (V - 35) >> 1 == chain_id, V >= 2^64 so no underflow
        uint32_t t[8];
        uint64_t br = 35;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const uint64_t d = (uint64_t)v[k] - br;
          t[k] = (uint32_t)d;
          br = (d >> 63) & 1;
        }
        bool hi0 = (t[2] >> 1) == 0;
#pragma unroll
        for (int k = 3; k < 8; ++k) hi0 = hi0 && t[k] == 0;
        const uint64_t sh = ((uint64_t)t[0] >> 1) | ((uint64_t)t[1] << 31) | ((uint64_t)(t[2] & 1u) << 63);
        match = hi0 && sh == chain_id;
      }
      if (!match) {
        status = ST_INVALID_CHAIN_ID;
      } else {
        // V' = V - 2*chainId - 8 (big.Int, no wrap)
        const uint64_t lo = chain_id * 2 + 8;
        const uint32_t hi = (uint32_t)((chain_id >> 63) & 1u) + (uint32_t)(chain_id * 2 + 8 < 8 ? 1 : 0);
        uint32_t sub[8] = {(uint32_t)lo, (uint32_t)(lo >> 32), hi, 0, 0, 0, 0, 0};
        uint64_t br = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const uint64_t d = (uint64_t)v[k] - sub[k] - br;
          vb8[k] = (uint32_t)d;
          br = (d >> 63) & 1;
        }
        vb_wide = false;
      }
    }
    homestead = true;
  }
  uint32_t recid = 0;
  if (status == ST_OK) {
    // recoverPlain :223-229
    if (vb_wide || bitlen_limbs(vb8) > 8) {
      status = ST_INVALID_SIG;
    } else {
      const uint32_t vv = (vb8[0] - 27u) & 0xffu;
      // ValidateSignatureValues (crypto.go:181-192)
      bool r_zero = true, s_zero = true;
#pragma unroll
      for (int k = 0; k < 8; ++k) { r_zero = r_zero && r[k] == 0; s_zero = s_zero && s[k] == 0; }
      const bool r_lt_1 = !r_wide && r_zero, s_lt_1 = !s_wide && s_zero;
      const bool s_high = s_wide || !u256_ge(SC_HALF, s);
      const bool r_ge_n = r_wide || u256_ge(r, SC_N), s_ge_n = s_wide || u256_ge(s, SC_N);
      if (r_lt_1 || s_lt_1 || (homestead && s_high) || r_ge_n || s_ge_n || !(vv == 0 || vv == 1))
        status = ST_INVALID_SIG;
      else
        recid = vv;
    }
  }
  return recid | (status << 8);
}

}  // namespace eges
