#pragma once
// types.Sender classification of one signature (transaction_signing.go:127-137,182-184,218-247,
// crypto.go:181-192, transaction.go:142-149, deriveChainId :250-260): items that fail before
// the C call get their Go error as status; the rest become ecrecover records with recid = v.
// Shared by prep_sender_kernel (k_prep.hip) and the fused wire-format mid-size kernel.
#include "core.cuh"
#include "rlp.cuh"

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

// The record lat_parse builds, from a sender row's little-endian limbs (z = the signing hash,
// r, s, v) and its vflags: prep_sender_kernel's classification and prep's range checks.
DEV LatParse sender_record(const uint32_t z[8], const uint32_t r[8], const uint32_t s[8], const uint32_t v[8],
                           uint32_t fl, int signer, uint64_t chain_id) {
  LatParse q;
  q.meta = sender_meta(r, s, v, fl, signer, chain_id);
  q.recid = q.meta & 3u;
  q.ok = ((q.meta >> 8) & 0xffu) == ST_OK;
  bool ovr, ovs, ovz;
  q.R = sc_from_limbs(r, ovr);
  q.Sv = sc_from_limbs(s, ovs);
  q.Z = sc_from_limbs(z, ovz);  // msg mod n (main_impl.h:183)
  q.ok = q.ok && !ovr && !ovs && !sc_is_zero(q.R) && !sc_is_zero(q.Sv);
#pragma unroll
  for (int i = 0; i < 8; ++i) q.xr[i] = q.R.v[i];  // recid < 2 on this path: x = r
  return q;
}

// Sender rows (RecoverParams::snd_*, 4-byte aligned) of item idx, one lane (root helpers, the
// mid-size kernel): eight dword loads per row, limb i = byte-swapped dword 7 - i.
DEV void row_limbs(uint32_t out[8], const uint8_t* row, uint32_t idx) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(row + (size_t)idx * 32);
#pragma unroll
  for (int i = 0; i < 8; ++i) out[i] = __builtin_bswap32(w[7 - i]);
}
DEV LatParse sender_parse_lane(const RecoverParams& prm, uint32_t idx) {
  uint32_t z[8], r[8], s[8], v[8];
  row_limbs(z, prm.snd_h, idx);
  row_limbs(r, prm.snd_r, idx);
  row_limbs(s, prm.snd_s, idx);
  row_limbs(v, prm.snd_v, idx);
  const uint32_t fl = prm.snd_f ? prm.snd_f[idx] : 0u;
  return sender_record(z, r, s, v, fl, prm.snd_signer, prm.snd_chain_id);
}
// The same for a whole wave working on one item (the latency kernels' row-form waves): one load
// instruction fetches the item's four rows (lane 8 k + j: dword j of row k) and its flags byte
// (lane 32); the limbs come back wave-uniform through readlane.
DEV LatParse sender_parse_wave(const RecoverParams& prm, uint32_t idx) {
  const uint32_t lane = (uint32_t)__lane_id();
  const uint32_t k = lane >> 3, j = lane & 7u;
  const uint8_t* row = k == 0 ? prm.snd_h : k == 1 ? prm.snd_r : k == 2 ? prm.snd_s : prm.snd_v;
  uint32_t w = 0;
  if (lane < 32) w = reinterpret_cast<const uint32_t*>(row + (size_t)idx * 32)[j];
  else if (lane == 32 && prm.snd_f) w = prm.snd_f[idx];
  uint32_t z[8], r[8], s[8], v[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    z[i] = __builtin_bswap32((uint32_t)__builtin_amdgcn_readlane((int)w, 7 - i));
    r[i] = __builtin_bswap32((uint32_t)__builtin_amdgcn_readlane((int)w, 15 - i));
    s[i] = __builtin_bswap32((uint32_t)__builtin_amdgcn_readlane((int)w, 23 - i));
    v[i] = __builtin_bswap32((uint32_t)__builtin_amdgcn_readlane((int)w, 31 - i));
  }
  const uint32_t fl = (uint32_t)__builtin_amdgcn_readlane((int)w, 32);
  return sender_record(z, r, s, v, fl, prm.snd_signer, prm.snd_chain_id);
}

// One wire-format transaction p[0, len) (span_ok: its offsets were consistent) -> the record
// lat_parse builds from rows (R, S, meta = recid | status << 8, R's x; z is left to the caller,
// who hashes m, the signing payload) — tx_rows_kernel's decode and prep_sender_kernel's
// classification in one: the fused wire paths of the mid-size and latency kernels. Returns
// whether the transaction decoded (m is valid only then).
DEV bool wire_item(const uint8_t* p, uint64_t len, bool span_ok, int signer, uint64_t chain_id, LatParse& q,
                   Payload& m) {
  RlpHead f[10]{};
  const bool ok = span_ok && tx_parse(p, len, signer, chain_id, f, m);
  uint32_t r[8], s[8], v[8];
  uint32_t fl = VF_DECODE_ERR;
  if (ok) {
    uint8_t b[32];
    fl = 0;
    fl |= rlp_to_be32(p, f[7], b) ? 0u : 1u;  // EGES_VF_V_WIDE
    limbs_from_be32(v, b);
    fl |= rlp_to_be32(p, f[8], b) ? 0u : 2u;  // EGES_VF_R_WIDE
    limbs_from_be32(r, b);
    fl |= rlp_to_be32(p, f[9], b) ? 0u : 4u;  // EGES_VF_S_WIDE
    limbs_from_be32(s, b);
  } else {
#pragma unroll
    for (int k = 0; k < 8; ++k) r[k] = s[k] = v[k] = 0;
  }
  const uint32_t z0[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // z: the caller hashes m
  q = sender_record(z0, r, s, v, fl, signer, chain_id);
  return ok;
}

}  // namespace eges
