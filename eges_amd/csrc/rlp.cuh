#pragma once
// RLP decode of the 10-field Geec txdata and its signing payload (device functions shared by
// tx_rows_kernel / tx_rows_wave_kernel, k_txhash.hip, and the fused wire-format form of the
// mid-size recover kernel, k_recover_mid.hip). The reference rules each function follows are
// cited in k_txhash.hip's header.
#include "core.cuh"

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
  h.b = p[size ? off : pos] & (size ? 0xffu : 0u);  // (both addresses inside the item: see Payload::at)
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
    const uint8_t b = p[j >= 0 ? src + j : h.start];  // in-bounds whichever way the select goes
    out[k] = j >= 0 ? b : (uint8_t)0;
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
  // The one memory read is at an index clamped into [mid0, mid0 + mid_len) (mid_len >= 1 for a
  // decoded txdata) whatever j is: when the compiler turns the branches into selects and loads
  // unconditionally, the address still lies inside the item. (Unclamped, a header byte j of a
  // payload whose header is longer than the transaction's, mid0 < hlen, became p[-1]: one byte
  // before the first encoding, an aperture violation when p is the start of a wave's LDS stage.)
  DEV uint32_t at(uint64_t j) const {
    const uint64_t k = j - hlen;  // wraps below hlen
    const uint64_t q = mid0 + (k < mid_len ? k : 0);
    const uint32_t mb = (to_patch && q == to_pos) ? 0x80u : (uint32_t)p[q];
    if (j < hlen) return j < 8 ? (uint32_t)(hdr0 >> (8 * j)) & 0xffu : (uint32_t)hdr1 & 0xffu;
    j -= hlen;
    if (j < mid_len) return mb;
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

}  // namespace eges
