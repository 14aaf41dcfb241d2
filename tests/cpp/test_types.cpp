// Tests of the host-side Go-layer mirror (include/eges_types.hpp), modelled on the reference's
// own tests of the same code: core/types/transaction_signing_test.go (signers, chain-id checks,
// the sender cache), transaction_test.go (RLP round trips), core/tx_pool_test.go
// (TestInvalidTransactions' ErrInvalidSender) and the block import loop. Driven by
// tests/test_types_host.py (mode `cpu`: no engine compute) and tests/test_gpu_types_host.py
// (mode `gpu`: every engine result against the fixture's oracle expectations).
//
//   test_types cpu <vectors.txt>   one hex tx per line -> "decode roundtrip protected hF hE"
//   test_types gpu <fixture.txt>   "tx <hex> <stE> <addrE> <stH> <addrH>" / "block <hex> <accepted> <n>"
// Every check prints one line; the exit status is the number of failed checks.
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "eges.h"
#include "eges_types.hpp"

using namespace eges;
using types::Address;
using types::Bytes;
using types::Err;
using types::Signer;
using types::Transaction;
using types::TxPtr;

static int g_fail = 0;
static void check(bool ok, const std::string& name, const std::string& detail = "") {
  std::printf("%s %s%s%s\n", ok ? "ok" : "FAIL", name.c_str(), detail.empty() ? "" : " : ", detail.c_str());
  if (!ok) ++g_fail;
}

static Bytes unhex(const std::string& h) {
  Bytes b(h.size() / 2);
  for (size_t i = 0; i < b.size(); ++i) b[i] = (uint8_t)std::stoi(h.substr(2 * i, 2), nullptr, 16);
  return b;
}
template <class C>
static std::string hex(const C& c) {
  static const char* d = "0123456789abcdef";
  std::string s;
  for (uint8_t x : c) {
    s += d[x >> 4];
    s += d[x & 15];
  }
  return s;
}
static int err_status(Err e) {  // Err -> EGES status byte (the fixture's encoding)
  switch (e) {
    case Err::kNone: return EGES_OK;
    case Err::kInvalidChainId: return EGES_INVALID_CHAIN_ID;
    case Err::kInvalidSig: return EGES_INVALID_SIG;
    case Err::kRecoverFailed: return EGES_RECOVER_FAILED;
    case Err::kDecode: return EGES_DECODE_FAILED;
    default: return -1;
  }
}

// ------------------------------------------------------------------ cpu mode
static TxPtr sample_tx(uint64_t nonce, uint8_t v) {
  types::TxData d;
  d.nonce = nonce;
  d.price = {0x01};
  d.gas = 21000;
  Address to;
  to.fill(0x42);
  d.to = to;
  d.amount = {0x0d, 0xe0};
  d.payload = Bytes(100, 0);
  d.v = {v};
  d.r = Bytes(32, 0x11);
  d.s = Bytes(32, 0x22);
  return std::make_shared<Transaction>(d);
}

static void cpu_unit() {
  // Signer.Equal (transaction_signing.go:120-123,170-173,197-200)
  const Signer F = Signer::Frontier(), H = Signer::Homestead(), E1 = Signer::EIP155(1), E2 = Signer::EIP155(2);
  check(F.Equal(F) && H.Equal(H) && E1.Equal(Signer::EIP155(1)), "signer equal: same type / chain id");
  check(!F.Equal(H) && !H.Equal(F) && !E1.Equal(E2) && !E1.Equal(H) && !H.Equal(E1) && !F.Equal(E1),
        "signer equal: different type or chain id");
  // MakeSigner (:42-53) over the fork blocks
  types::ChainConfig geec;  // chain 930412, Homestead and EIP-155 at 0
  check(Signer::Make(geec, 0).Equal(Signer::EIP155(930412)), "MakeSigner: Geec genesis -> EIP155(930412)");
  types::ChainConfig c2;
  c2.chain_id = 7;
  c2.homestead_block = 5;
  c2.eip155_block = 10;
  check(Signer::Make(c2, 4).Equal(F) && Signer::Make(c2, 5).Equal(H) && Signer::Make(c2, 9).Equal(H) &&
            Signer::Make(c2, 10).Equal(Signer::EIP155(7)),
        "MakeSigner: Frontier / Homestead / EIP155 by block number");
  c2.eip155_block.reset();
  check(Signer::Make(c2, 1000).Equal(H), "MakeSigner: no EIP-155 fork -> Homestead");
  // the pool's signer is types.NewEIP155Signer(chainconfig.ChainId) (tx_pool.go:227) whatever
  // the fork schedule and head: protected transactions stay acceptable before the fork block
  check(core::TxPool(c2, 1000).signer().Equal(Signer::EIP155(7)) && core::TxPool(c2, 0).signer().Equal(Signer::EIP155(7)),
        "TxPool signer: EIP155(chain id) with the EIP-155 fork unset");
  c2.eip155_block = 10;
  check(core::TxPool(c2, 4).signer().Equal(Signer::EIP155(7)), "TxPool signer: EIP155(chain id) below the fork block");
  // isProtectedV (transaction.go:142-149)
  check(!sample_tx(0, 27)->Protected() && !sample_tx(0, 28)->Protected() && sample_tx(0, 37)->Protected() &&
            sample_tx(0, 0)->Protected(),
        "Protected: 27/28 unprotected, 37 and 0 protected");
  // the sender cache (transaction_signing.go:72-89): a cached sender under an Equal signer is
  // returned without any engine call; a non-Equal signer misses (and, with no device here, the
  // engine call fails and the cache keeps its entry)
  const TxPtr tx = sample_tx(3, 37);
  Address a;
  a.fill(0xab);
  tx->StoreFrom(Signer::EIP155(1), a);
  const uint64_t c0 = types::EngineCalls();
  Address got{};
  Err e = types::Sender(Signer::EIP155(1), *tx, &got);
  check(e == Err::kNone && got == a && types::EngineCalls() == c0, "Sender: cache hit under an Equal signer");
  std::vector<Err> errs;
  e = types::RecoverSenders(Signer::EIP155(1), {tx, tx}, &errs);
  check(e == Err::kNone && errs.size() == 2 && errs[0] == Err::kNone && types::EngineCalls() == c0,
        "RecoverSenders: all cached -> no engine call");
  if (eges_device_count() == 0 && eges_init(0, 0) != EGES_SUCCESS) {
    e = types::Sender(Signer::EIP155(2), *tx, &got);
    check(e == Err::kEngine && types::EngineCalls() == c0 + 1, "Sender: a non-Equal signer misses the cache",
          types::ErrString(e));
    auto c = tx->CachedFrom();
    check(c && c->signer.Equal(Signer::EIP155(1)) && c->from == a, "Sender: a failed call leaves the cache");
  }
  // RLP round trip of a constructed transaction
  Err de;
  const TxPtr back = Transaction::Decode(tx->rlp().data(), tx->rlp().size(), &de);
  check(back && de == Err::kNone && back->rlp() == tx->rlp() && back->data().nonce == 3 && back->data().gas == 21000 &&
            back->data().to && (*back->data().to)[0] == 0x42 && back->data().payload.size() == 100,
        "EncodeRLP / DecodeRLP round trip");
}

static int cpu_mode(const char* path) {
  cpu_unit();
  std::ifstream in(path);
  std::string line;
  while (std::getline(in, line)) {
    if (line.empty()) continue;
    const Bytes raw = unhex(line);
    Err e;
    const TxPtr tx = Transaction::Decode(raw.data(), raw.size(), &e);
    if (!tx) {
      std::printf("vec 0 0 0 - -\n");
      continue;
    }
    const auto hf = Signer::Frontier().Hash(*tx);
    const auto he = Signer::EIP155(930412).Hash(*tx);
    std::printf("vec 1 %d %d %s %s\n", tx->rlp() == raw ? 1 : 0, tx->Protected() ? 1 : 0, hex(hf).c_str(),
                hex(he).c_str());
  }
  return g_fail;
}

// ------------------------------------------------------------------ gpu mode
struct Item {
  Bytes raw;
  int st_e, st_h;
  Address a_e, a_h;
};

static std::vector<TxPtr> fresh(const std::vector<Item>& items) {
  std::vector<TxPtr> v;
  for (const Item& it : items) {
    Err e;
    v.push_back(Transaction::Decode(it.raw.data(), it.raw.size(), &e));
  }
  return v;
}

static int gpu_mode(const char* path) {
  if (eges_init(0, 0) != EGES_SUCCESS) {
    check(false, "eges_init", eges_last_error());
    return g_fail;
  }
  std::ifstream in(path);
  std::string line;
  std::vector<Item> items;
  struct Blk {
    Bytes raw;
    int accepted;
    size_t n;
  };
  std::vector<Blk> blocks;
  while (std::getline(in, line)) {
    std::istringstream ss(line);
    std::string kind, h;
    ss >> kind >> h;
    if (kind == "tx") {
      Item it;
      std::string ae, ah;
      ss >> it.st_e >> ae >> it.st_h >> ah;
      it.raw = unhex(h);
      const Bytes be = unhex(ae), bh = unhex(ah);
      std::memcpy(it.a_e.data(), be.data(), 20);
      std::memcpy(it.a_h.data(), bh.data(), 20);
      items.push_back(it);
    } else if (kind == "block") {
      Blk b;
      ss >> b.accepted >> b.n;
      b.raw = unhex(h);
      blocks.push_back(b);
    }
  }
  const size_t n = items.size();
  const Signer E = Signer::EIP155(930412), H = Signer::Homestead();
  std::vector<TxPtr> txs = fresh(items);
  bool decoded = true;
  for (const TxPtr& t : txs) decoded = decoded && t;
  check(decoded && n > 0, "fixture transactions decode", std::to_string(n));
  if (!decoded) return g_fail;

  // 1. RecoverSenders: one engine call, every outcome the oracle's
  uint64_t c0 = types::EngineCalls();
  std::vector<Err> errs;
  Err rc = types::RecoverSenders(E, txs, &errs);
  size_t bad = 0;
  for (size_t i = 0; i < n; ++i) {
    Address a{};
    const Err e2 = types::Sender(E, *txs[i], &a);  // cached on success; a recomputation otherwise
    if (err_status(errs[i]) != items[i].st_e || err_status(e2) != items[i].st_e) ++bad;
    else if (items[i].st_e == EGES_OK && !(a == items[i].a_e)) ++bad;
  }
  size_t n_bad_e = 0;
  for (const Item& it : items) n_bad_e += it.st_e != EGES_OK;
  check(rc == Err::kNone && bad == 0, "RecoverSenders(EIP155) == oracle, item for item", std::to_string(bad));
  // the per-tx Sender loop after the batch: cache hits, except the failing items (not cached)
  check(types::EngineCalls() - c0 == 1 + n_bad_e, "RecoverSenders: one call; later Sender calls hit the cache",
        std::to_string(types::EngineCalls() - c0));

  // 2. another signer misses the cache and re-derives (Homestead on EIP-155 V: ErrInvalidSig)
  rc = types::RecoverSenders(H, txs, &errs);
  bad = 0;
  for (size_t i = 0; i < n; ++i) {
    if (err_status(errs[i]) != items[i].st_h) ++bad;
    else if (items[i].st_h == EGES_OK) {
      auto c = txs[i]->CachedFrom();
      if (!c || !c->signer.Equal(H) || !(c->from == items[i].a_h)) ++bad;
    }
  }
  check(rc == Err::kNone && bad == 0, "RecoverSenders(Homestead) == oracle; cache re-keyed", std::to_string(bad));

  // 3. the reference's per-tx path: one Sender (one engine call) per transaction, fresh objects
  std::vector<TxPtr> t2 = fresh(items);
  c0 = types::EngineCalls();
  bad = 0;
  const size_t m = std::min<size_t>(n, 96);
  for (size_t i = 0; i < m; ++i) {
    Address a{};
    const Err e = types::Sender(E, *t2[i], &a);
    if (err_status(e) != items[i].st_e || (e == Err::kNone && !(a == items[i].a_e))) ++bad;
  }
  check(bad == 0 && types::EngineCalls() - c0 == m, "Sender per tx (single-item path) == oracle", std::to_string(bad));

  // 4. tx pool ingress: batched addTxsLocked vs the per-tx loop, same outcomes
  std::vector<TxPtr> t3 = fresh(items), t4 = fresh(items);
  core::TxPool pool(types::ChainConfig{}), ref(types::ChainConfig{});
  ref.batch = false;
  c0 = types::EngineCalls();
  const auto pe = pool.AddRemotes(t3);
  const uint64_t calls_batch = types::EngineCalls() - c0;
  c0 = types::EngineCalls();
  const auto pr = ref.AddRemotes(t4);
  const uint64_t calls_ref = types::EngineCalls() - c0;
  bad = 0;
  size_t n_ok = 0;
  for (size_t i = 0; i < n; ++i) {
    const core::PoolErr want = items[i].st_e == EGES_OK ? core::PoolErr::kNone : core::PoolErr::kInvalidSender;
    if (pe[i] != want || pr[i] != want) ++bad;
    n_ok += want == core::PoolErr::kNone;
  }
  check(bad == 0 && pool.PendingCount() == n_ok && ref.PendingCount() == n_ok,
        "TxPool.AddRemotes: ErrInvalidSender exactly where types.Sender fails (batched == per-tx)",
        std::to_string(bad));
  check(calls_ref == n && calls_batch == 1, "TxPool: one engine call per batch instead of one per tx",
        std::to_string(calls_batch) + " vs " + std::to_string(calls_ref));
  bool same_pending = pool.Pending().size() == ref.Pending().size();
  for (const auto& kv : pool.Pending()) {
    auto it = ref.Pending().find(kv.first);
    same_pending = same_pending && it != ref.Pending().end() && it->second.size() == kv.second.size();
  }
  check(same_pending, "TxPool: pending sets by sender identical");
  const auto again = pool.AddRemotes(t3);
  bad = 0;
  for (size_t i = 0; i < n; ++i)
    if (again[i] != (items[i].st_e == EGES_OK ? core::PoolErr::kKnown : core::PoolErr::kInvalidSender)) ++bad;
  check(bad == 0, "TxPool: re-added transactions are known", std::to_string(bad));
  // journal replay (tx_pool.go:243): the loaded list as one batch
  core::TxPool jp(types::ChainConfig{});
  const auto je = jp.LoadJournal(fresh(items));
  bad = 0;
  for (size_t i = 0; i < n; ++i) bad += je[i] != pe[i];
  check(bad == 0 && jp.PendingCount() == n_ok, "TxPool.LoadJournal: journal replay as one batch");

  // 5. block import: Process's sender loop behind one RecoverSenders
  core::Block blk;
  std::vector<size_t> good;
  for (size_t i = 0; i < n; ++i)
    if (items[i].st_e == EGES_OK) good.push_back(i);
  std::vector<TxPtr> t5 = fresh(items);
  for (size_t i : good) blk.txs.push_back(t5[i]);
  c0 = types::EngineCalls();
  auto pr5 = core::ProcessSenders(types::ChainConfig{}, blk);
  bad = pr5.senders.size() != good.size();
  for (size_t k = 0; !bad && k < good.size(); ++k) bad += !(pr5.senders[k] == items[good[k]].a_e);
  check(pr5.err == Err::kNone && bad == 0 && types::EngineCalls() - c0 == 1,
        "ProcessSenders: block senders in order, one engine call");
  if (n_bad_e) {
    size_t first_bad = 0;
    while (items[first_bad].st_e == EGES_OK) ++first_bad;
    core::Block b2;
    b2.txs = fresh(items);
    auto r2 = core::ProcessSenders(types::ChainConfig{}, b2);
    core::Block b3;
    b3.txs = fresh(items);
    c0 = types::EngineCalls();
    auto r3 = core::ProcessSenders(types::ChainConfig{}, b3, false);
    check(types::EngineCalls() - c0 == first_bad + 1, "ProcessSenders per tx: one engine call per tx up to the failure");
    check(r2.failed == first_bad && err_status(r2.err) == items[first_bad].st_e && r3.failed == r2.failed &&
              r3.err == r2.err && r2.senders.size() == first_bad,
          "ProcessSenders: stops at the first failing tx with its error (batched == per-tx)");
  }

  // 6. the Geec validator hook over whole blocks
  for (size_t k = 0; k < blocks.size(); ++k) {
    const auto v = core::GeecValidate(types::ChainConfig{}, 1, blocks[k].raw.data(), blocks[k].raw.size());
    check((v.accepted ? 1 : 0) == blocks[k].accepted && (blocks[k].accepted == 0 || v.senders.size() == blocks[k].n),
          "GeecValidate block " + std::to_string(k), std::to_string(v.accepted) + " status " + std::to_string(v.block_status));
  }
  return g_fail;
}

int main(int argc, char** argv) {
  if (argc < 3) {
    std::fprintf(stderr, "usage: test_types cpu|gpu <file>\n");
    return 2;
  }
  const std::string mode = argv[1];
  const int f = mode == "cpu" ? cpu_mode(argv[2]) : gpu_mode(argv[2]);
  std::printf("failed %d\n", f);
  return f ? 1 : 0;
}
