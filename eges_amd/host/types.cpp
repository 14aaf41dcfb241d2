// Host-side mirror of core/types' sender path (include/eges_types.hpp): Transaction with its
// sender cache, the three signers, types.Sender and the batch RecoverSenders over libeges.so.
#include <algorithm>
#include <atomic>
#include <cstring>

#include "eges.h"
#include "eges_types.hpp"

namespace eges {
namespace types {

namespace {

std::atomic<uint64_t> g_engine_calls{0};

// ---------------------------------------------------------------- RLP encoding (rlp/encode.go)
void put_len(Bytes& o, size_t n, uint8_t off) {
  if (n < 56) {
    o.push_back((uint8_t)(off + n));
    return;
  }
  uint8_t be[8];
  int k = 0;
  for (size_t x = n; x; x >>= 8) be[k++] = (uint8_t)x;
  o.push_back((uint8_t)(off + 55 + k));
  while (k) o.push_back(be[--k]);
}
void enc_string(Bytes& o, const uint8_t* p, size_t n) {
  if (n == 1 && p[0] < 0x80) {
    o.push_back(p[0]);
    return;
  }
  put_len(o, n, 0x80);
  o.insert(o.end(), p, p + n);
}
void enc_string(Bytes& o, const Bytes& b) { enc_string(o, b.data(), b.size()); }
void enc_uint(Bytes& o, uint64_t x) {
  uint8_t be[8];
  int k = 0;
  for (; x; x >>= 8) be[k++] = (uint8_t)x;
  uint8_t buf[8];
  for (int i = 0; i < k; ++i) buf[i] = be[k - 1 - i];
  enc_string(o, buf, (size_t)k);
}
Bytes wrap_list(const Bytes& body) {
  Bytes o;
  put_len(o, body.size(), 0xC0);
  o.insert(o.end(), body.begin(), body.end());
  return o;
}
// the first six txdata fields, shared by the wire form and the signing payloads
void enc_common(Bytes& o, const TxData& d) {
  enc_uint(o, d.nonce);
  enc_string(o, d.price);
  enc_uint(o, d.gas);
  if (d.to) enc_string(o, d.to->data(), 20);
  else o.push_back(0x80);  // nil *common.Address with rlp:"nil"
  enc_string(o, d.amount);
  enc_string(o, d.payload);
}

// ---------------------------------------------------------------- RLP decoding (rlp/decode.go)
// Restates the acceptance rules the reference decoder applies to the Geec txdata struct (the
// same rules oracle/txoracle.py and the GPU decoder k_txhash.hip apply): canonical sizes and
// integers, uint64 overflow, booleans, [20]byte recipients with rlp:"nil", too few / too many
// list elements, no trailing bytes.
struct Stream {
  const uint8_t* b;
  size_t pos, end;
  bool ok = true;
  bool eol = false;  // the list ended before a field: "too few elements"

  bool byte(uint8_t& x) {
    if (pos >= end) return false;
    x = b[pos++];
    return true;
  }
  bool uint_be(size_t n, uint64_t& v) {
    v = 0;
    if (n == 0) return true;
    uint8_t first;
    if (!byte(first)) return false;
    if (n > 1 && first == 0) return false;  // ErrCanonSize
    v = first;
    for (size_t i = 1; i < n; ++i) {
      uint8_t x;
      if (!byte(x)) return false;
      v = (v << 8) | x;
    }
    return true;
  }
  // header -> kind 0 byte (value in `bv`), 1 string, 2 list, with the content size
  bool kind(int& k, size_t& size, uint8_t& bv) {
    if (pos == end) {
      eol = true;
      return false;
    }
    uint8_t h;
    if (!byte(h)) return false;
    uint64_t sz = 0;
    if (h < 0x80) {
      k = 0;
      bv = h;
      size = 0;
      return true;
    } else if (h < 0xB8) {
      k = 1;
      sz = h - 0x80;
    } else if (h < 0xC0) {
      if (!uint_be(h - 0xB7u, sz) || sz < 56) return false;
      k = 1;
    } else if (h < 0xF8) {
      k = 2;
      sz = h - 0xC0;
    } else {
      if (!uint_be(h - 0xF7u, sz) || sz < 56) return false;
      k = 2;
    }
    if (sz > end - pos) return false;  // ErrElemTooLarge / ErrValueTooLarge
    size = (size_t)sz;
    return true;
  }
  bool bytes(Bytes& out) {
    int k;
    size_t size;
    uint8_t bv;
    if (!kind(k, size, bv)) return false;
    if (k == 0) {
      out.assign(1, bv);
      return true;
    }
    if (k == 2) return false;  // ErrExpectedString
    out.assign(b + pos, b + pos + size);
    pos += size;
    return !(size == 1 && out[0] < 0x80);  // ErrCanonSize
  }
  bool uint(unsigned maxbits, uint64_t& v) {
    int k;
    size_t size;
    uint8_t bv;
    if (!kind(k, size, bv)) return false;
    if (k == 0) {
      v = bv;
      return bv != 0;  // ErrCanonInt
    }
    if (k == 2 || size > maxbits / 8) return false;
    if (size >= 2 && b[pos] == 0) return false;  // ErrCanonInt
    v = 0;
    for (size_t i = 0; i < size; ++i) v = (v << 8) | b[pos + i];
    pos += size;
    return !(size > 0 && v < 128);  // ErrCanonSize
  }
  bool bigint(Bytes& out) {
    if (!bytes(out)) return false;
    return out.empty() || out[0] != 0;  // ErrCanonInt
  }
  bool boolean(bool& x) {
    uint64_t v;
    if (!uint(8, v) || v > 1) return false;
    x = v == 1;
    return true;
  }
  bool address_or_nil(std::optional<Address>& to) {
    int k;
    size_t size;
    uint8_t bv;
    if (!kind(k, size, bv)) return false;
    if (size == 0 && k != 0) {
      to.reset();
      return true;
    }
    if (k == 0 || k == 2 || size != 20) return false;  // [20]byte: too short / long, not a string
    Address a;
    std::memcpy(a.data(), b + pos, 20);
    pos += 20;
    to = a;
    return true;
  }
};

bool decode_txdata(const uint8_t* raw, size_t len, TxData& d) {
  Stream s{raw, 0, len};
  int k;
  size_t size;
  uint8_t bv;
  if (!s.kind(k, size, bv) || k != 2) return false;  // ErrExpectedList
  const size_t list_end = s.pos + size;
  s.end = list_end;
  const bool fields = s.uint(64, d.nonce) && s.bigint(d.price) && s.uint(64, d.gas) && s.address_or_nil(d.to) &&
                      s.bigint(d.amount) && s.bytes(d.payload) && s.boolean(d.is_geec) && s.bigint(d.v) &&
                      s.bigint(d.r) && s.bigint(d.s);
  if (!fields) return false;         // including "too few elements"
  if (s.pos != list_end) return false;  // "input list has too many elements"
  return list_end == len;            // ErrMoreThanOneValue
}

Bytes encode_txdata(const TxData& d) {
  Bytes body;
  enc_common(body, d);
  body.push_back(d.is_geec ? 0x01 : 0x80);
  enc_string(body, d.v);
  enc_string(body, d.r);
  enc_string(body, d.s);
  return wrap_list(body);
}

Err err_of_status(uint8_t st) {
  switch (st) {
    case EGES_OK: return Err::kNone;
    case EGES_INVALID_CHAIN_ID: return Err::kInvalidChainId;
    case EGES_INVALID_SIG: return Err::kInvalidSig;
    case EGES_DECODE_FAILED: return Err::kDecode;
    default: return Err::kRecoverFailed;
  }
}

}  // namespace

const char* ErrString(Err e) {
  switch (e) {
    case Err::kNone: return "ok";
    case Err::kInvalidChainId: return "invalid chain id for signer";
    case Err::kInvalidSig: return "invalid transaction v, r, s values";
    case Err::kRecoverFailed: return "recovery failed";
    case Err::kDecode: return "rlp: invalid transaction encoding";
    case Err::kEngine: return "sender engine call failed";
  }
  return "?";
}

uint64_t EngineCalls() { return g_engine_calls.load(); }

// ---------------------------------------------------------------- Signer
Signer Signer::Frontier() { return Signer(EGES_SIGNER_FRONTIER, 0); }
Signer Signer::Homestead() { return Signer(EGES_SIGNER_HOMESTEAD, 0); }
Signer Signer::EIP155(uint64_t chain_id) { return Signer(EGES_SIGNER_EIP155, chain_id); }

Signer Signer::Make(const ChainConfig& cfg, uint64_t number) {
  if (cfg.eip155_block && *cfg.eip155_block <= number) return EIP155(cfg.chain_id);
  if (cfg.homestead_block && *cfg.homestead_block <= number) return Homestead();
  return Frontier();
}

bool Signer::Equal(const Signer& o) const {
  if (kind_ != o.kind_) return false;
  return kind_ != EGES_SIGNER_EIP155 || chain_id_ == o.chain_id_;
}

Hash32 Signer::Hash(const Transaction& tx) const {
  Bytes body;
  enc_common(body, tx.data());
  if (kind_ == EGES_SIGNER_EIP155) {  // s.chainId, uint(0), uint(0)
    enc_uint(body, chain_id_);
    body.push_back(0x80);
    body.push_back(0x80);
  }
  const Bytes l = wrap_list(body);
  Hash32 h;
  eges_keccak256(l.data(), l.size(), h.data());
  return h;
}

// ---------------------------------------------------------------- Transaction
Transaction::Transaction(TxData d) : d_(std::move(d)), enc_(encode_txdata(d_)) {}

std::shared_ptr<Transaction> Transaction::Decode(const uint8_t* raw, size_t len, Err* err) {
  TxData d;
  if (!raw || !decode_txdata(raw, len, d)) {
    if (err) *err = Err::kDecode;
    return nullptr;
  }
  if (err) *err = Err::kNone;
  return std::make_shared<Transaction>(std::move(d));
}

bool Transaction::Protected() const {
  const Bytes& v = d_.v;  // isProtectedV: V.BitLen() <= 8 -> v != 27 && v != 28; else true
  if (v.size() <= 1) {
    const unsigned x = v.empty() ? 0u : v[0];
    return x != 27 && x != 28;
  }
  return true;
}

std::shared_ptr<const Transaction::SigCache> Transaction::CachedFrom() const { return std::atomic_load(&from_); }

void Transaction::StoreFrom(const Signer& s, const Address& from) const {
  std::atomic_store(&from_, std::shared_ptr<const SigCache>(new SigCache{s, from}));
}

// ---------------------------------------------------------------- Sender / RecoverSenders
namespace {
// signer.Sender over the given transactions' wire forms: one eges_sender_raw_batch call
Err engine_senders(const Signer& s, const std::vector<const Transaction*>& txs, std::vector<uint8_t>& st,
                   std::vector<uint8_t>& addr) {
  const size_t n = txs.size();
  st.assign(n, 0);
  addr.assign(n * 20, 0);
  if (!n) return Err::kNone;
  size_t total = 0;
  for (const Transaction* t : txs) total += t->rlp().size();
  Bytes raw;
  raw.reserve(total);
  std::vector<uint64_t> off(n + 1);
  for (size_t i = 0; i < n; ++i) {
    off[i] = raw.size();
    raw.insert(raw.end(), txs[i]->rlp().begin(), txs[i]->rlp().end());
  }
  off[n] = raw.size();
  g_engine_calls.fetch_add(1);
  const int rc = eges_sender_raw_batch(raw.data(), off.data(), n, s.kind(), s.chain_id(), addr.data(), st.data(), nullptr);
  return rc == EGES_SUCCESS ? Err::kNone : Err::kEngine;
}
}  // namespace

Err Sender(const Signer& s, const Transaction& tx, Address* out) {
  if (auto c = tx.CachedFrom(); c && c->signer.Equal(s)) {
    if (out) *out = c->from;
    return Err::kNone;
  }
  std::vector<uint8_t> st, addr;
  const Err e = engine_senders(s, {&tx}, st, addr);
  if (e != Err::kNone) return e;
  const Err r = err_of_status(st[0]);
  if (r != Err::kNone) return r;
  Address a;
  std::memcpy(a.data(), addr.data(), 20);
  tx.StoreFrom(s, a);
  if (out) *out = a;
  return Err::kNone;
}

Err RecoverSenders(const Signer& s, const std::vector<TxPtr>& txs, std::vector<Err>* errs) {
  std::vector<Err> e(txs.size(), Err::kNone);
  std::vector<const Transaction*> miss;
  std::vector<size_t> at;
  for (size_t i = 0; i < txs.size(); ++i) {
    auto c = txs[i]->CachedFrom();
    if (c && c->signer.Equal(s)) continue;
    miss.push_back(txs[i].get());
    at.push_back(i);
  }
  std::vector<uint8_t> st, addr;
  const Err rc = engine_senders(s, miss, st, addr);
  if (rc != Err::kNone) {
    if (errs) errs->assign(txs.size(), rc);
    return rc;
  }
  for (size_t k = 0; k < miss.size(); ++k) {
    e[at[k]] = err_of_status(st[k]);
    if (st[k] == EGES_OK) {
      Address a;
      std::memcpy(a.data(), &addr[k * 20], 20);
      miss[k]->StoreFrom(s, a);
    }
  }
  if (errs) *errs = std::move(e);
  return Err::kNone;
}

}  // namespace types
}  // namespace eges
