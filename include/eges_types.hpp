// Host-side mirror of the reference's Go layer above the cgo seam, in C++ (no Go toolchain in
// this build image): the parts of core/types and core that decide which transactions reach
// crypto.Ecrecover, rewired onto libeges.so's batch entries.
//
//   types::Transaction ........ core/types/transaction.go:50-76 (txdata, the `from` cache :56),
//                               DecodeRLP / EncodeRLP :157-165, isProtectedV :142-149
//   types::Signer ............. transaction_signing.go:91-220 (Frontier / Homestead / EIP155,
//                               Equal, Hash), MakeSigner :42-53
//   types::Sender ............. transaction_signing.go:72-89 (the sigCache lookup keyed by
//                               Signer.Equal; on a miss signer.Sender, then the cache store)
//   types::RecoverSenders ..... new: the batch that fills every cache of a list in one engine call
//                               
//   core::TxPool .............. tx_pool.go:800-830 addTxs / addTxsLocked with validateTx's sender
//                               check (:570-574, ErrInvalidSender), journal replay (:243,
//                               tx_journal.go:59): one RecoverSenders before the per-tx loop
//   core::ProcessSenders ...... state_processor.go:73-93 (Process -> ApplyTransaction -> AsMessage
//                               -> types.Sender) behind blockchain.go:1219's insertChain: one
//                               RecoverSenders per block before the serial loop
//   core::GeecValidate ........ core/geec_state.go:528-550 (Validate accepts every block today):
//                               the block's signed transactions recovered in one call
//
// Everything that is not signature work (state, gas, nonces, balances, promotion) is out of
// scope; the mirrors keep only the sender decisions and their error mapping, so
// that a batch prefetch can be checked to leave every per-transaction outcome unchanged.
#pragma once

#include <array>
#include <cstddef>
#include <cstdint>
#include <map>
#include <memory>
#include <optional>
#include <string>
#include <vector>

namespace eges {
namespace types {

using Bytes = std::vector<uint8_t>;
using Address = std::array<uint8_t, 20>;
using Hash32 = std::array<uint8_t, 32>;

// Errors a sender derivation can end in (one per Go error value it can return).
enum class Err : int {
  kNone = 0,
  kInvalidChainId,  // types.ErrInvalidChainId      transaction_signing.go:30-32
  kInvalidSig,      // types.ErrInvalidSig          transaction.go:36 (recoverPlain :223-229)
  kRecoverFailed,   // secp256k1.ErrRecoverFailed   crypto/secp256k1/secp256.go:61
  kDecode,          // an rlp error of DecodeRLP    transaction.go:157-165, rlp/decode.go
  kEngine,          // the engine call itself failed (eges_last_error(); no device, ...)
};
const char* ErrString(Err e);

// params.ChainConfig's fork fields used by MakeSigner (params/config.go IsHomestead / IsEIP155).
// Geec's genesis: chain id 930412, Homestead and EIP-155 at block 0 (genesis.json.template:3-5).
struct ChainConfig {
  uint64_t chain_id = 930412;
  std::optional<uint64_t> homestead_block = 0;
  std::optional<uint64_t> eip155_block = 0;
};

// txdata (transaction.go:59-76). big.Ints are held as canonical big-endian bytes (no leading
// zero byte; empty means 0), exactly what their RLP strings carry.
struct TxData {
  uint64_t nonce = 0;
  Bytes price;
  uint64_t gas = 0;
  std::optional<Address> to;  // nil: contract creation
  Bytes amount;
  Bytes payload;
  bool is_geec = false;
  Bytes v, r, s;
};

class Transaction;

class Signer {
 public:
  static Signer Frontier();
  static Signer Homestead();
  static Signer EIP155(uint64_t chain_id);
  static Signer Make(const ChainConfig& cfg, uint64_t block_number);  // MakeSigner :42-53
  // EIP155Signer.Equal :120-123 (same chain id), HomesteadSigner.Equal :170-173,
  // FrontierSigner.Equal :197-200 (same type)
  bool Equal(const Signer& o) const;
  int kind() const { return kind_; }  // EGES_SIGNER_*
  uint64_t chain_id() const { return chain_id_; }
  // Hash(tx): EIP155Signer.Hash :155-165, FrontierSigner.Hash :207-216 (Homestead inherits it)
  Hash32 Hash(const Transaction& tx) const;

 private:
  Signer(int kind, uint64_t chain_id) : kind_(kind), chain_id_(chain_id) {}
  int kind_;
  uint64_t chain_id_;
};

class Transaction {
 public:
  explicit Transaction(TxData d);  // the txdata of NewTransaction + WithSignature
  // rlp.DecodeBytes(raw, tx) with the reference decoder's rules for txdata; null + *err on error
  static std::shared_ptr<Transaction> Decode(const uint8_t* raw, size_t len, Err* err);
  const TxData& data() const { return d_; }
  const Bytes& rlp() const { return enc_; }  // EncodeRLP (canonical; the bytes Decode accepted)
  bool Protected() const;                   // isProtectedV(V) :142-149
  // The sender cache (tx.from atomic.Value :56 holding a sigCache :36-39).
  struct SigCache {
    Signer signer;
    Address from;
  };
  std::shared_ptr<const SigCache> CachedFrom() const;         // tx.from.Load()
  void StoreFrom(const Signer& s, const Address& from) const;  // tx.from.Store(sigCache{...})

 private:
  TxData d_;
  Bytes enc_;
  mutable std::shared_ptr<const SigCache> from_;  // accessed only through std::atomic_load/store
};
using TxPtr = std::shared_ptr<Transaction>;

// types.Sender: the cached address when the cached signer Equals `s`; otherwise signer.Sender(tx)
// through the engine (one item), then the cache store on success.
Err Sender(const Signer& s, const Transaction& tx, Address* out);

// Every transaction of `txs` whose cache misses under `s` recovered in ONE engine call
// (eges_sender_raw_batch: GPU decode, sighash, V rules, recovery); caches filled on success.
// errs[i] is exactly what Sender(s, *txs[i]) would return. Returns kEngine (and leaves the
// caches untouched) when the engine call fails.
Err RecoverSenders(const Signer& s, const std::vector<TxPtr>& txs, std::vector<Err>* errs);

// Engine-call counter (tests: a cache hit must not reach the engine).
uint64_t EngineCalls();

}  // namespace types

namespace core {

// tx_pool.go:46-90 error values the sender check maps to.
enum class PoolErr : int {
  kNone = 0,
  kInvalidSender,  // ErrInvalidSender (validateTx :570-574: any types.Sender error)
  kKnown,          // ErrKnownTransaction-style duplicate of a pending (sender, nonce) (pool.add)
  kEngine,
};

// The pool's ingress with only its sender decisions: addTxs / addTxsLocked (tx_pool.go:800-830)
// run one RecoverSenders under the pool lock, then the unchanged per-tx loop (validateTx's
// types.Sender now hits the cache). Accepted transactions are kept per sender by nonce.
class TxPool {
 public:
  // head_number does not pick the signer: the pool always uses EIP155(cfg.chain_id) (tx_pool.go:227)
  explicit TxPool(const types::ChainConfig& cfg, uint64_t head_number = 0);
  std::vector<PoolErr> AddRemotes(const std::vector<types::TxPtr>& txs);  // AddRemotes -> addTxs(false)
  std::vector<PoolErr> AddLocals(const std::vector<types::TxPtr>& txs);   // AddLocals -> addTxs(true)
  // journal replay (tx_pool.go:243 journal.load(pool.AddLocal), tx_journal.go:59-94): the loaded
  // transactions in one batch instead of one AddLocal (and one Sender) each
  std::vector<PoolErr> LoadJournal(const std::vector<types::TxPtr>& txs);
  size_t PendingCount() const;
  const std::map<types::Address, std::map<uint64_t, types::TxPtr>>& Pending() const { return pending_; }
  const types::Signer& signer() const { return signer_; }
  bool batch = true;  // false: the reference's per-tx path (each Sender a separate engine call)

 private:
  std::vector<PoolErr> AddTxsLocked(const std::vector<types::TxPtr>& txs, bool local);
  types::Signer signer_;
  std::map<types::Address, std::map<uint64_t, types::TxPtr>> pending_;
};

// A block as insertChain sees it (core/types/block.go): number + transactions.
struct Block {
  uint64_t number = 0;
  std::vector<types::TxPtr> txs;
};

// StateProcessor.Process's sender loop (state_processor.go:73-93: ApplyTransaction -> AsMessage ->
// types.Sender with MakeSigner(config, header.Number)), preceded by one RecoverSenders of the
// block (blockchain.go:1219, before bc.processor.Process). Returns the senders in block order,
// or the first failing transaction's index and error (Process stops there).
struct ProcessResult {
  types::Err err = types::Err::kNone;
  size_t failed = 0;
  std::vector<types::Address> senders;
};
ProcessResult ProcessSenders(const types::ChainConfig& cfg, const Block& b, bool batch = true);

// GeecState.Validate (core/geec_state.go:528-550) with the signature check the reference lacks:
// the proposed block (extblock RLP) in one eges_block_senders_raw call over its Txs; accepted when
// the block decodes and every transaction recovers a sender under MakeSigner.
struct ValidateResult {
  bool accepted = false;
  int block_status = 0;        // EGES_OK / EGES_DECODE_FAILED
  std::vector<uint8_t> status; // per Txs item
  std::vector<types::Address> senders;
};
ValidateResult GeecValidate(const types::ChainConfig& cfg, uint64_t number, const uint8_t* block_rlp, size_t len);

}  // namespace core
}  // namespace eges
