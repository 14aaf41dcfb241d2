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

#include <cstdlib>

namespace eges {

enum : int { RK_BYTE = 0, RK_STRING = 1, RK_LIST = 2 };

struct RlpHead {
  int kind;
  uint64_t start; // first byte of the item (its header)
  uint64_t off;   // first content byte (Byte kind: the byte itself)
  uint64_t size;  // content bytes (0 for Byte)
  uint64_t next;  // position after the item
  uint32_t b;     // Byte kind: the value; String: first content byte (if size > 0)
};

// Head of the item at pos inside [pos, lim). false on any error the reference's Stream.Kind
// reports there (EOF / EOL, non-canonical size, element larger than the containing list).
DEV bool rlp_head(const uint8_t* __restrict__ p, uint64_t pos, uint64_t lim, RlpHead& h) {
  if (pos >= lim) return false;
  h.start = pos;
  const uint32_t b0 = p[pos];
  if (b0 < 0x80u) {
    h.kind = RK_BYTE;
    h.off = pos;
    h.size = 0;
    h.next = pos + 1;
    h.b = b0;
    return true;
  }
  uint64_t size, off;
  if (b0 < 0xB8u || (b0 >= 0xC0u && b0 < 0xF8u)) {
    size = b0 < 0xB8u ? b0 - 0x80u : b0 - 0xC0u;
    off = pos + 1;
  } else {
    const uint32_t ll = b0 < 0xC0u ? b0 - 0xB7u : b0 - 0xF7u;  // 1..8 length bytes
    if (lim - pos - 1 < ll) return false;
    if (ll >= 2 && p[pos + 1] == 0) return false;  // leading zero in the size: ErrCanonSize
    size = 0;
    for (uint32_t k = 0; k < ll; ++k) size = (size << 8) | p[pos + 1 + k];
    if (size < 56) return false;  // long form for a short item: ErrCanonSize
    off = pos + 1 + ll;
  }
  if (size > lim - off) return false;  // ErrElemTooLarge / ErrValueTooLarge
  h.kind = b0 < 0xC0u ? RK_STRING : RK_LIST;
  h.off = off;
  h.size = size;
  h.next = off + size;
  h.b = size ? p[off] : 0u;
  return true;
}

// Stream.uint(bits) acceptance (uint64 nonce / gas: bits 64; bool: bits 8, value checked apart).
DEV bool rlp_uint_ok(const RlpHead& h, uint32_t max_bytes) {
  if (h.kind == RK_BYTE) return h.b != 0;  // a single 0x00 byte: ErrCanonInt
  if (h.kind != RK_STRING) return false;   // ErrExpectedString
  if (h.size > max_bytes) return false;    // errUintOverflow
  if (h.size == 1) return h.b >= 0x80u;    // should have been a single byte: ErrCanonSize
  if (h.size >= 2) return h.b != 0;        // leading zero: ErrCanonInt
  return true;
}
// decodeBigInt: Bytes() then the leading-zero rule.
DEV bool rlp_bigint_ok(const RlpHead& h) {
  if (h.kind == RK_BYTE) return h.b != 0;
  if (h.kind != RK_STRING) return false;
  if (h.size == 1 && h.b < 0x80u) return false;
  if (h.size > 0 && h.b == 0) return false;
  return true;
}
// decodeByteSlice (Payload)
DEV bool rlp_bytes_ok(const RlpHead& h) {
  if (h.kind == RK_BYTE) return true;
  if (h.kind != RK_STRING) return false;
  return !(h.size == 1 && h.b < 0x80u);
}

// Big-endian integer content -> 32-byte left-padded row; returns false if wider than 256 bits.
DEV bool rlp_to_be32(const uint8_t* __restrict__ p, const RlpHead& h, uint8_t* __restrict__ out) {
  const uint64_t len = h.kind == RK_BYTE ? 1 : h.size;
  if (len > 32) {
    for (int k = 0; k < 32; ++k) out[k] = 0;
    return false;
  }
  const uint64_t src = h.off;
  for (int k = 0; k < 32; ++k) {
    const int j = k - (32 - (int)len);
    out[k] = j >= 0 ? p[src + j] : (uint8_t)0;
  }
  return true;
}

// The signing payload as a byte stream: hdr (<= 9 bytes) || raw[mid0, mid0 + mid_len) with
// raw[to_pos] replaced by 0x80 when `to` is nil || tail (<= 11 bytes).
struct Payload {
  const uint8_t* p;
  uint64_t hdr0, hdr1;  // header bytes, little-endian packed
  uint32_t hlen;
  uint64_t mid0, mid_len, to_pos;
  bool to_patch;
  uint64_t tail0, tail1;
  uint32_t tlen;
  DEV uint32_t at(uint64_t j) const {
    if (j < hlen) return j < 8 ? (uint32_t)(hdr0 >> (8 * j)) & 0xffu : (uint32_t)hdr1 & 0xffu;
    j -= hlen;
    if (j < mid_len) {
      const uint64_t q = mid0 + j;
      return (to_patch && q == to_pos) ? 0x80u : (uint32_t)p[q];
    }
    j -= mid_len;
    if (j < tlen) return j < 8 ? (uint32_t)(tail0 >> (8 * j)) & 0xffu : (uint32_t)(tail1 >> (8 * (j - 8))) & 0xffu;
    return 0;
  }
  DEV uint64_t length() const { return hlen + mid_len + tlen; }
};

// Keccak-256 sponge (rate 136, domain byte 0x01: sha3.NewKeccak256, crypto/sha3/hashes.go:16).
DEV void keccak256_payload(const Payload& m, uint8_t* __restrict__ out32) {
  uint64_t A[25];
#pragma unroll
  for (int i = 0; i < 25; ++i) A[i] = 0;
  const uint64_t M = m.length();
  const uint64_t nblk = M / 136 + 1;
#pragma unroll 1
  for (uint64_t b = 0; b < nblk; ++b) {
    const uint64_t base = b * 136;
#pragma unroll
    for (int w = 0; w < 17; ++w) {
      uint64_t x = 0;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const uint64_t j = base + 8 * w + k;
        uint64_t byte = j < M ? m.at(j) : 0u;
        if (j == M) byte ^= 0x01u;
        if (b + 1 == nblk && 8 * w + k == 135) byte ^= 0x80u;
        x |= byte << (8 * k);
      }
      A[w] ^= x;
    }
    keccak_f1600(A);
  }
#pragma unroll
  for (int i = 0; i < 32; ++i) out32[i] = (uint8_t)(A[i >> 3] >> (8 * (i & 7)));
}

// rlp encoding of a uint64 (rlp/encode.go writeUint): packed little-endian bytes, returns length.
DEV uint32_t enc_uint(uint64_t v, uint64_t& lo, uint64_t& hi) {
  if (v == 0) {
    lo = 0x80;
    hi = 0;
    return 1;
  }
  if (v < 0x80) {
    lo = v;
    hi = 0;
    return 1;
  }
  const uint32_t nb = (64 - __clzll(v) + 7) / 8;
  uint8_t b[9];
  b[0] = (uint8_t)(0x80 + nb);
  for (uint32_t k = 0; k < 8; ++k) b[1 + k] = k < nb ? (uint8_t)(v >> (8 * (nb - 1 - k))) : 0;
  lo = 0;
  for (int k = 0; k < 8; ++k) lo |= (uint64_t)b[k] << (8 * k);
  hi = b[8];
  return 1 + nb;
}

// Decode one txdata held in p[0, lim) and build its signing payload (steps 1 and 2 above).
// false on a decode error. f[7..9] are the V, R, S items.
DEV bool tx_parse(const uint8_t* __restrict__ p, uint64_t lim, int signer, uint64_t chain_id, RlpHead f[10],
                  Payload& m) {
  RlpHead L{};
  bool ok = rlp_head(p, 0, lim, L) && L.kind == RK_LIST && L.next == lim;  // one value, no trailer
  uint64_t pos = L.off;
  const uint64_t lend = L.off + L.size;
#pragma unroll
  for (int k = 0; k < 10; ++k) {
    ok = ok && rlp_head(p, pos, lend, f[k]);  // pos == lend: too few elements
    pos = ok ? f[k].next : pos;
  }
  ok = ok && pos == lend;  // too many elements
  ok = ok && rlp_uint_ok(f[0], 8) && rlp_bigint_ok(f[1]) && rlp_uint_ok(f[2], 8);
  // Recipient *common.Address `rlp:"nil"`: empty string or empty list -> nil, else exactly 20 bytes
  const bool to_nil = f[3].kind != RK_BYTE && f[3].size == 0;
  ok = ok && (to_nil || (f[3].kind == RK_STRING && f[3].size == 20));
  ok = ok && rlp_bigint_ok(f[4]) && rlp_bytes_ok(f[5]);
  // IsGeecTxn bool: 0x80 (false) or 0x01 (true)
  ok = ok && ((f[6].kind == RK_BYTE && f[6].b == 1u) || (f[6].kind == RK_STRING && f[6].size == 0));
  ok = ok && rlp_bigint_ok(f[7]) && rlp_bigint_ok(f[8]) && rlp_bigint_ok(f[9]);
  if (!ok) return false;
  // isProtectedV (transaction.go:142-149): V.BitLen() <= 8 && V in {27, 28} is unprotected
  const uint64_t vlen = f[7].kind == RK_BYTE ? 1 : f[7].size;
  const uint32_t v0 = vlen == 0 ? 0u : f[7].b;
  const bool prot = vlen <= 1 ? !(v0 == 27u || v0 == 28u) : true;
  const bool eip155 = signer == 2 && prot;
  m.p = p;
  m.mid0 = f[0].start;                  // nonce .. payload items, as received
  m.mid_len = f[6].start - f[0].start;  // up to the IsGeecTxn item
  m.to_pos = f[3].start;                // nil `to` is the single byte 0x80 or 0xC0
  m.to_patch = to_nil;
  m.tlen = 0;
  m.tail0 = m.tail1 = 0;
  if (eip155) {
    uint64_t lo, hi;
    const uint32_t cl = enc_uint(chain_id, lo, hi);
    // chainId || uint(0) || uint(0)
    uint8_t t[11];
    for (int k = 0; k < 11; ++k) t[k] = 0;
    for (uint32_t k = 0; k < cl; ++k) t[k] = k < 8 ? (uint8_t)(lo >> (8 * k)) : (uint8_t)hi;
    t[cl] = 0x80;
    t[cl + 1] = 0x80;
    m.tlen = cl + 2;
    for (int k = 0; k < 8; ++k) m.tail0 |= (uint64_t)t[k] << (8 * k);
    for (int k = 8; k < 11; ++k) m.tail1 |= (uint64_t)t[k] << (8 * (k - 8));
  }
  const uint64_t body = m.mid_len + m.tlen;
  if (body < 56) {
    m.hdr0 = 0xC0 + body;
    m.hdr1 = 0;
    m.hlen = 1;
  } else {
    const uint32_t nb = (64 - __clzll(body) + 7) / 8;
    uint8_t h[9];
    h[0] = (uint8_t)(0xF7 + nb);
    for (uint32_t k = 0; k < 8; ++k) h[1 + k] = k < nb ? (uint8_t)(body >> (8 * (nb - 1 - k))) : 0;
    m.hdr0 = 0;
    for (int k = 0; k < 8; ++k) m.hdr0 |= (uint64_t)h[k] << (8 * k);
    m.hdr1 = h[8];
    m.hlen = 1 + nb;
  }
  return true;
}

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
  return (len <= 32 && j >= 0) ? p[h.off + j] : 0u;
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
  // KNOB_TXROWS_WAVE_MAX (default 8192, capi.hip) sets the cut (0: never the wave form)
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
