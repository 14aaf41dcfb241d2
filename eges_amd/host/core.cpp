// Host-side mirror of the core call sites that derive senders (include/eges_types.hpp): the tx
// pool's ingress and journal replay, the block processor's sender loop behind insertChain, and
// the Geec validator hook. Each keeps the reference's per-transaction decision and error mapping
// and puts one batch engine call in front of it.
#include <cstring>

#include "eges.h"
#include "eges_types.hpp"

namespace eges {
namespace core {

using types::Address;
using types::Err;
using types::Signer;
using types::TxPtr;

// ---------------------------------------------------------------- TxPool
// pool.signer = types.NewEIP155Signer(chainconfig.ChainId) (tx_pool.go:227), whatever the fork
// schedule and the head: the pool accepts EIP-155-protected transactions before the fork block
TxPool::TxPool(const types::ChainConfig& cfg, uint64_t head_number) : signer_(Signer::EIP155(cfg.chain_id)) {
  (void)head_number;
}

std::vector<PoolErr> TxPool::AddRemotes(const std::vector<TxPtr>& txs) { return AddTxsLocked(txs, false); }
std::vector<PoolErr> TxPool::AddLocals(const std::vector<TxPtr>& txs) { return AddTxsLocked(txs, true); }
std::vector<PoolErr> TxPool::LoadJournal(const std::vector<TxPtr>& txs) { return AddTxsLocked(txs, true); }

size_t TxPool::PendingCount() const {
  size_t n = 0;
  for (const auto& kv : pending_) n += kv.second.size();
  return n;
}

// addTxsLocked (tx_pool.go:809-822): for each tx, pool.add -> known check, validateTx's
// `types.Sender(pool.signer, tx)` (:570-574, any error -> ErrInvalidSender), insertion. With
// `batch`, one RecoverSenders fills every cache first, so the loop's Sender calls all hit.
std::vector<PoolErr> TxPool::AddTxsLocked(const std::vector<TxPtr>& txs, bool local) {
  (void)local;  // locals skip the price floor only, which is not a signature decision
  std::vector<PoolErr> out(txs.size(), PoolErr::kNone);
  std::vector<Err> errs;  // the batch's verdicts: a failed derivation is not cached, so the loop
                          // takes its error from here instead of deriving it a second time
  if (batch && types::RecoverSenders(signer_, txs, &errs) == Err::kEngine) {
    out.assign(txs.size(), PoolErr::kEngine);
    return out;
  }
  for (size_t i = 0; i < txs.size(); ++i) {
    const TxPtr& tx = txs[i];
    Address from{};
    const Err e = batch && errs[i] != Err::kNone ? errs[i] : types::Sender(signer_, *tx, &from);
    if (e == Err::kEngine) {
      out[i] = PoolErr::kEngine;
      continue;
    }
    if (e != Err::kNone) {
      out[i] = PoolErr::kInvalidSender;
      continue;
    }
    auto& acct = pending_[from];
    auto it = acct.find(tx->data().nonce);
    if (it != acct.end() && it->second->rlp() == tx->rlp()) {
      out[i] = PoolErr::kKnown;  // pool.add: "known transaction"
      continue;
    }
    acct[tx->data().nonce] = tx;
  }
  return out;
}

// ---------------------------------------------------------------- block import
ProcessResult ProcessSenders(const types::ChainConfig& cfg, const Block& b, bool batch) {
  ProcessResult r;
  const Signer s = Signer::Make(cfg, b.number);  // types.MakeSigner(p.config, header.Number)
  std::vector<Err> errs;
  if (batch && types::RecoverSenders(s, b.txs, &errs) == Err::kEngine) {
    r.err = Err::kEngine;
    return r;
  }
  r.senders.reserve(b.txs.size());
  for (size_t i = 0; i < b.txs.size(); ++i) {  // for i, tx := range block.Transactions()
    Address a{};
    // tx.AsMessage(signer) -> types.Sender (a cache hit after the batch, or the batch's error)
    const Err e = batch && errs[i] != Err::kNone ? errs[i] : types::Sender(s, *b.txs[i], &a);
    if (e != Err::kNone) {
      r.err = e;
      r.failed = i;
      return r;
    }
    r.senders.push_back(a);
  }
  return r;
}

// ---------------------------------------------------------------- Geec validator
ValidateResult GeecValidate(const types::ChainConfig& cfg, uint64_t number, const uint8_t* block_rlp, size_t len) {
  ValidateResult v;
  const Signer s = Signer::Make(cfg, number);
  uint32_t counts[3] = {0, 0, 0};
  int bst = 0;
  // first call sizes the Txs list (cap 0 rejects any non-empty list with EGES_E_INVALID_ARG, but
  // still reports the counts and the structure status)
  int rc = eges_block_senders_raw(block_rlp, len, EGES_LIST_TXS, s.kind(), s.chain_id(), 0, nullptr, nullptr, counts, &bst);
  if (rc != EGES_SUCCESS && rc != EGES_E_INVALID_ARG) return v;
  v.block_status = bst;
  if (bst != EGES_OK) return v;  // undecodable block: rejected
  const size_t n = counts[2];
  std::vector<uint8_t> addr(n * 20 + 20), st(n + 1);
  rc = eges_block_senders_raw(block_rlp, len, EGES_LIST_TXS, s.kind(), s.chain_id(), n, addr.data(), st.data(), counts, &bst);
  if (rc != EGES_SUCCESS) return v;
  v.block_status = bst;
  v.status.assign(st.begin(), st.begin() + n);
  v.accepted = bst == EGES_OK;
  for (size_t i = 0; i < n; ++i) {
    Address a;
    std::memcpy(a.data(), &addr[i * 20], 20);
    v.senders.push_back(a);
    if (st[i] != EGES_OK) v.accepted = false;
  }
  return v;
}

}  // namespace core
}  // namespace eges
