// Host-side AddressSanitizer + UBSan run of libeges. The library is rebuilt
// with the sanitizers on its HOST code only (`make -C eges_amd/csrc asan`: -Xarch_host
// -fsanitize=...; device code is not instrumented, GPU ASan is not available on this pool) and
// this driver links it. Without a GPU it exercises every host-only path: argument validation of
// each C-ABI entry, the host Keccak against known answers, the Geec block splitter on
// well-formed, truncated and randomly mutated blocks, and the single-item coalescer's error path
// from several threads. With a GPU (eges_init succeeds) it adds the data paths: batch recovery
// through the chunked and the pinned small-call lanes, single-item recover / verify from 8
// threads through the coalescer, a signed Geec block through eges_block_senders_raw and
// eges_sender_raw_batch, eges_sender_batch, the precompile and batch verify, every result checked
// against the synthetic signer's expected address. Exit 0 = no sanitizer report, no mismatch.
//   build: make -C eges_amd/csrc asan   (-> tools/asan/{libeges_asan.so,sanitize_host})
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "eges.h"

using bytes = std::vector<uint8_t>;
static long g_checks = 0, g_fail = 0;
#define CHECK(c, ...)                                             \
  do {                                                            \
    ++g_checks;                                                   \
    if (!(c)) {                                                   \
      ++g_fail;                                                   \
      std::fprintf(stderr, "MISMATCH %s:%d: ", __FILE__, __LINE__); \
      std::fprintf(stderr, __VA_ARGS__);                          \
      std::fputc('\n', stderr);                                   \
    }                                                             \
  } while (0)

static uint64_t g_rng = 0x2545f4914f6cdd1dull;
static uint64_t rnd() {
  g_rng ^= g_rng << 13;
  g_rng ^= g_rng >> 7;
  g_rng ^= g_rng << 17;
  return g_rng;
}

// ---- RLP encoding (rlp/encode.go rules), enough to build transactions and extblocks
static bytes rlp_len(size_t n, uint8_t off) {
  if (n < 56) return {uint8_t(off + n)};
  bytes be;
  for (size_t x = n; x; x >>= 8) be.insert(be.begin(), uint8_t(x));
  be.insert(be.begin(), uint8_t(off + 55 + be.size()));
  return be;
}
static bytes rlp_bytes(const bytes& b) {
  if (b.size() == 1 && b[0] < 0x80) return b;
  bytes r = rlp_len(b.size(), 0x80);
  r.insert(r.end(), b.begin(), b.end());
  return r;
}
static bytes be_trim(const uint8_t* p, size_t n) {
  size_t i = 0;
  while (i < n && p[i] == 0) ++i;
  return bytes(p + i, p + n);
}
static bytes rlp_uint(uint64_t x) {
  uint8_t b[8];
  for (int i = 0; i < 8; ++i) b[i] = uint8_t(x >> (56 - 8 * i));
  return rlp_bytes(be_trim(b, 8));
}
static bytes rlp_list(const std::vector<bytes>& items) {
  bytes body;
  for (auto& x : items) body.insert(body.end(), x.begin(), x.end());
  bytes r = rlp_len(body.size(), 0xC0);
  r.insert(r.end(), body.begin(), body.end());
  return r;
}

static const uint64_t CHAIN = 930412;  // genesis.json.template:3-5
static const bytes TO(20, 0x22);

// 10-field Geec txdata (core/types/transaction.go:59-76)
static bytes geec_tx(uint64_t nonce, const bytes& data, bool is_geec, uint64_t v, const bytes& r, const bytes& s) {
  return rlp_list({rlp_uint(nonce), rlp_uint(1), rlp_uint(21000), rlp_bytes(TO), rlp_uint(7), rlp_bytes(data),
                   bytes{uint8_t(is_geec ? 0x01 : 0x80)}, rlp_uint(v), rlp_bytes(r), rlp_bytes(s)});
}
// EIP155Signer.Hash (transaction_signing.go:155-165)
static void eip155_hash(uint64_t nonce, const bytes& data, uint8_t out[32]) {
  bytes m = rlp_list({rlp_uint(nonce), rlp_uint(1), rlp_uint(21000), rlp_bytes(TO), rlp_uint(7), rlp_bytes(data),
                      rlp_uint(CHAIN), rlp_uint(0), rlp_uint(0)});
  eges_keccak256(m.data(), m.size(), out);
}
static bytes header() {
  return rlp_list({rlp_bytes(bytes(32, 0)), rlp_bytes(bytes(32, 0x1d)), rlp_bytes(bytes(20, 0x11)), rlp_uint(1),
                   rlp_uint(8000000), rlp_list({}), rlp_uint(7)});
}
static bytes extblock(const std::vector<bytes>& fake, const std::vector<bytes>& geec, const std::vector<bytes>& txs) {
  return rlp_list({header(), rlp_list(fake), rlp_list(geec), rlp_list(txs), rlp_list({}), rlp_list({})});
}

// ---- host-only paths
static void keccak_known_answers() {
  static const uint8_t empty[32] = {0xc5, 0xd2, 0x46, 0x01, 0x86, 0xf7, 0x23, 0x3c, 0x92, 0x7e, 0x7d,
                                    0xb2, 0xdc, 0xc7, 0x03, 0xc0, 0xe5, 0x00, 0xb6, 0x53, 0xca, 0x82,
                                    0x27, 0x3b, 0x7b, 0xfa, 0xd8, 0x04, 0x5d, 0x85, 0xa4, 0x70};
  uint8_t h[32], h2[32];
  eges_keccak256(nullptr, 0, h);
  CHECK(!std::memcmp(h, empty, 32), "keccak(\"\")");
  // every length over two rate boundaries, exact-size heap buffers
  for (size_t len = 1; len <= 2 * 136 + 3; ++len) {
    uint8_t* in = static_cast<uint8_t*>(std::malloc(len));
    for (size_t i = 0; i < len; ++i) in[i] = uint8_t(rnd());
    eges_keccak256(in, len, h);
    eges_keccak256(in, len, h2);
    CHECK(!std::memcmp(h, h2, 32), "keccak deterministic %zu", len);
    std::free(in);
  }
}

static void argument_validation() {
  uint8_t b[256] = {0};
  uint64_t off[2] = {0, 0};
  uint32_t counts[3];
  int bst;
  CHECK(eges_ecrecover_batch(nullptr, b, 1, b, b, b) != EGES_SUCCESS, "NULL msg");
  CHECK(eges_ecrecover_batch(b, b, 0, nullptr, nullptr, nullptr) == EGES_SUCCESS, "n = 0");
  CHECK(eges_sender_batch(b, b, b, b, b, 1, 7, 1, b, b) != EGES_SUCCESS, "bad signer");
  CHECK(eges_sender_raw_batch(b, nullptr, 1, 2, 1, b, b, nullptr) != EGES_SUCCESS, "NULL offsets");
  CHECK(eges_sender_raw_batch(b, off, 0, 2, 1, b, b, nullptr) == EGES_SUCCESS, "raw n = 0");
  CHECK(eges_block_senders_raw(nullptr, 0, 7, 2, 1, 0, nullptr, nullptr, counts, &bst) != EGES_SUCCESS, "NULL block");
  CHECK(eges_block_senders_raw(b, 1, 7, 3, 1, 0, nullptr, nullptr, counts, &bst) != EGES_SUCCESS, "block bad signer");
  CHECK(eges_verify_batch(b, nullptr, b, b, 1, b) != EGES_SUCCESS, "NULL publen");
  CHECK(eges_ecrecover_precompile_batch(nullptr, nullptr, 1, b, b) != EGES_SUCCESS, "NULL input");
  CHECK(eges_ecrecover_batch_dev(99, b, b, 1, b, b, b, nullptr) != EGES_SUCCESS, "bad device");
  CHECK(eges_last_error() && std::strlen(eges_last_error()) > 0, "error text");
  CHECK(eges_abi_version() == EGES_ABI_VERSION, "abi");
}

// The splitter on well-formed blocks, every strict prefix of one, and random byte mutations
// (lists = 0: structure and counts on the host; a structurally well-formed block's lists are
// then decode-checked on the GPU, so without a device its answer is EGES_E_NODEVICE).
static bool g_nodev = false;  // no HIP device visible (host-only run)

static void block_structure(int mutations) {
  std::vector<bytes> fake, geec, txs;
  for (int i = 0; i < 5; ++i) fake.push_back(geec_tx(0, bytes(100, 0), false, 0, {}, {}));
  for (int i = 0; i < 3; ++i) geec.push_back(geec_tx(0, bytes(23, 0x41), true, 0, {}, {}));
  for (int i = 0; i < 40; ++i) txs.push_back(geec_tx(i, bytes(i % 70), false, 37, bytes(32, 0x11), bytes(32, 0x22)));
  const bytes blk = extblock(fake, geec, txs);
  uint32_t counts[3];
  int bst = -1;
  const int rc0 = eges_block_senders_raw(blk.data(), blk.size(), 0, 2, CHAIN, 0, nullptr, nullptr, counts, &bst);
  CHECK((rc0 == EGES_SUCCESS || (g_nodev && rc0 == EGES_E_NODEVICE)) && bst == EGES_OK && counts[0] == 5 &&
            counts[1] == 3 && counts[2] == 40,
        "well-formed counts %u %u %u (rc %d)", counts[0], counts[1], counts[2], rc0);
  const bytes empty = extblock({}, {}, {});
  CHECK(eges_block_senders_raw(empty.data(), empty.size(), 7, 2, CHAIN, 0, nullptr, nullptr, counts, &bst) ==
                EGES_SUCCESS &&
            bst == EGES_OK && !counts[0] && !counts[1] && !counts[2],
        "empty block");
  for (size_t len = 0; len < blk.size(); ++len) {
    uint8_t* p = static_cast<uint8_t*>(std::malloc(len ? len : 1));  // exact size: overreads trap
    std::memcpy(p, blk.data(), len);
    bst = -1;
    const int rc = eges_block_senders_raw(len ? p : blk.data(), len, 0, 2, CHAIN, 0, nullptr, nullptr, counts, &bst);
    CHECK(rc == EGES_SUCCESS && bst == EGES_DECODE_FAILED, "prefix %zu accepted", len);
    std::free(p);
  }
  long accepted = 0;
  for (int m = 0; m < mutations; ++m) {
    bytes b = blk;
    const int k = 1 + int(rnd() % 4);
    for (int j = 0; j < k; ++j) {
      const size_t at = rnd() % b.size();
      switch (rnd() % 3) {
        case 0: b[at] = uint8_t(rnd()); break;
        case 1: b.erase(b.begin() + long(at)); break;
        default: b.insert(b.begin() + long(at), uint8_t(rnd())); break;
      }
    }
    uint8_t* p = static_cast<uint8_t*>(std::malloc(b.size()));
    std::memcpy(p, b.data(), b.size());
    bst = -1;
    const int rc = eges_block_senders_raw(p, b.size(), 0, 2, CHAIN, 0, nullptr, nullptr, counts, &bst);
    // a structurally well-formed block still needs the GPU decoder for its lists: without a
    // device that is EGES_E_NODEVICE (no CPU fallback), never a silent accept
    CHECK((rc == EGES_SUCCESS && (bst == EGES_OK || bst == EGES_DECODE_FAILED)) ||
              (g_nodev && rc == EGES_E_NODEVICE && bst == EGES_OK),
          "mutation rc %d bst %d", rc, bst);
    accepted += bst == EGES_OK;
    std::free(p);
  }
  std::printf("block splitter: %zu prefixes rejected, %d mutations (%ld still well-formed)\n", blk.size(), mutations,
              accepted);
}

// Single-item entries with no engine: the coalescer's failure path from several threads.
static void coalescer_without_device() {
  std::vector<std::thread> th;
  std::atomic<int> ok{0};
  for (int t = 0; t < 4; ++t)
    th.emplace_back([&] {
      uint8_t pub[65], sig[65] = {1}, msg[32] = {2};
      for (int k = 0; k < 50; ++k) ok += eges_ecdsa_recover(pub, sig, msg) == 1;
    });
  for (auto& x : th) x.join();
  CHECK(ok.load() == 0, "recover without a device succeeded");
}

// ---- data paths (GPU present)
struct Signed {
  bytes msg, sig, addr;
};
static Signed synth(uint64_t first, size_t n, const uint8_t* msg_in = nullptr) {
  uint8_t *dm, *ds, *da;
  Signed s{bytes(n * 32), bytes(n * 65), bytes(n * 20)};
  if (hipMalloc(&dm, n * 32) || hipMalloc(&ds, n * 65) || hipMalloc(&da, n * 20)) std::abort();
  if (msg_in) {
    if (hipMemcpy(dm, msg_in, n * 32, hipMemcpyHostToDevice)) std::abort();
    if (eges_synth_sign_msg_dev(0, first, n, dm, ds, da, nullptr) != EGES_SUCCESS) std::abort();
  } else if (eges_synth_sign_dev(0, first, n, dm, ds, da, nullptr) != EGES_SUCCESS) {
    std::abort();
  }
  if (hipDeviceSynchronize() || hipMemcpy(s.msg.data(), dm, n * 32, hipMemcpyDeviceToHost) ||
      hipMemcpy(s.sig.data(), ds, n * 65, hipMemcpyDeviceToHost) ||
      hipMemcpy(s.addr.data(), da, n * 20, hipMemcpyDeviceToHost))
    std::abort();
  (void)hipFree(dm), (void)hipFree(ds), (void)hipFree(da);
  return s;
}

static void batch_recover(size_t n) {
  const Signed s = synth(100000 + n, n);
  bytes pub(n * 65), addr(n * 20), st(n);
  CHECK(eges_ecrecover_batch(s.msg.data(), s.sig.data(), n, pub.data(), addr.data(), st.data()) == EGES_SUCCESS,
        "batch %zu: %s", n, eges_last_error());
  size_t bad = 0;
  for (size_t i = 0; i < n; ++i) bad += st[i] != EGES_OK || std::memcmp(&addr[i * 20], &s.addr[i * 20], 20);
  CHECK(bad == 0, "batch %zu: %zu wrong", n, bad);
  // verify the same signatures against the recovered keys; every 5th message altered
  bytes publen(n, 65), sig64(n * 64), msg = s.msg, ok(n);
  for (size_t i = 0; i < n; ++i) {
    std::memcpy(&sig64[i * 64], &s.sig[i * 65], 64);
    if (i % 5 == 0) msg[i * 32] ^= 1;
  }
  CHECK(eges_verify_batch(pub.data(), publen.data(), msg.data(), sig64.data(), n, ok.data()) == EGES_SUCCESS,
        "verify %zu", n);
  bad = 0;
  for (size_t i = 0; i < n; ++i) bad += ok[i] != (i % 5 != 0);
  CHECK(bad == 0, "verify %zu: %zu wrong", n, bad);
  // the precompile over the same items (hash, v = 27 + recid, r, s), every 7th input short
  bytes in(n * 128, 0), out(n * 32), pst(n);
  std::vector<uint32_t> inlen(n, 128);
  for (size_t i = 0; i < n; ++i) {
    std::memcpy(&in[i * 128], &s.msg[i * 32], 32);
    in[i * 128 + 63] = uint8_t(27 + s.sig[i * 65 + 64]);
    std::memcpy(&in[i * 128 + 64], &s.sig[i * 65], 64);
    if (i % 7 == 3) inlen[i] = uint32_t(rnd() % 128);
  }
  CHECK(eges_ecrecover_precompile_batch(in.data(), inlen.data(), n, out.data(), pst.data()) == EGES_SUCCESS,
        "precompile %zu", n);
  bad = 0;
  for (size_t i = 0; i < n; ++i)
    if (inlen[i] == 128) bad += pst[i] != EGES_OK || std::memcmp(&out[i * 32 + 12], &s.addr[i * 20], 20);
  CHECK(bad == 0, "precompile %zu: %zu wrong", n, bad);
}

static void single_item_threads(int threads, int calls) {
  const size_t n = 512;
  const Signed s = synth(777000, n);
  std::atomic<long> bad{0};
  std::vector<std::thread> th;
  for (int t = 0; t < threads; ++t)
    th.emplace_back([&, t] {
      for (int k = 0; k < calls; ++k) {
        const size_t i = size_t(t * 131 + k * 17) % n;
        uint8_t pub[65], h[32];
        if (eges_ecdsa_recover(pub, &s.sig[i * 65], &s.msg[i * 32]) != 1) {
          ++bad;
          continue;
        }
        eges_keccak256(pub + 1, 64, h);
        if (std::memcmp(h + 12, &s.addr[i * 20], 20)) ++bad;
        if (k % 4 == 0 && eges_ecdsa_verify(&s.sig[i * 65], &s.msg[i * 32], pub, 65) != 1) ++bad;
      }
    });
  for (auto& x : th) x.join();
  CHECK(bad.load() == 0, "single-item threads: %ld wrong", bad.load());
}

static void signed_block(size_t n) {
  std::vector<bytes> data(n);
  bytes sighash(n * 32);
  for (size_t i = 0; i < n; ++i) {
    data[i] = bytes(i % 130, uint8_t(i));
    eip155_hash(5000 + i, data[i], &sighash[i * 32]);
  }
  const Signed s = synth(5000, n, sighash.data());
  std::vector<bytes> txs, fake;
  bytes raw;
  std::vector<uint64_t> offs{0};
  for (size_t i = 0; i < n; ++i) {
    const uint8_t* sg = &s.sig[i * 65];
    txs.push_back(geec_tx(5000 + i, data[i], i % 3 == 0, sg[64] + 35 + 2 * CHAIN, be_trim(sg, 32),
                          be_trim(sg + 32, 32)));
    raw.insert(raw.end(), txs.back().begin(), txs.back().end());
    offs.push_back(raw.size());
  }
  for (int i = 0; i < 7; ++i) fake.push_back(geec_tx(0, bytes(100, 0), false, 0, {}, {}));
  const bytes blk = extblock(fake, {}, txs);
  bytes addr(n * 20), st(n), sh(n * 32);
  CHECK(eges_sender_raw_batch(raw.data(), offs.data(), n, 2, CHAIN, addr.data(), st.data(), sh.data()) ==
            EGES_SUCCESS,
        "raw batch: %s", eges_last_error());
  size_t bad = 0;
  for (size_t i = 0; i < n; ++i)
    bad += st[i] != EGES_OK || std::memcmp(&addr[i * 20], &s.addr[i * 20], 20) ||
           std::memcmp(&sh[i * 32], &sighash[i * 32], 32);
  CHECK(bad == 0, "raw batch: %zu wrong", bad);
  const size_t cap = n + 7;
  bytes baddr(cap * 20), bst_items(cap);
  uint32_t counts[3];
  int bst = -1;
  CHECK(eges_block_senders_raw(blk.data(), blk.size(), 7, 2, CHAIN, cap, baddr.data(), bst_items.data(), counts,
                               &bst) == EGES_SUCCESS,
        "block: %s", eges_last_error());
  CHECK(bst == EGES_OK && counts[0] == 7 && counts[1] == 0 && counts[2] == n, "block counts");
  bad = 0;
  for (size_t i = 0; i < 7; ++i) bad += bst_items[i] != EGES_INVALID_CHAIN_ID;
  for (size_t i = 0; i < n; ++i)
    bad += bst_items[7 + i] != EGES_OK || std::memcmp(&baddr[(7 + i) * 20], &s.addr[i * 20], 20);
  CHECK(bad == 0, "block items: %zu wrong", bad);
  CHECK(eges_block_senders_raw(blk.data(), blk.size(), 7, 2, CHAIN, cap - 1, baddr.data(), bst_items.data(), counts,
                               &bst) == EGES_E_INVALID_ARG,
        "cap too small accepted");
  // eges_sender_batch on the split fields
  bytes r(n * 32, 0), sv(n * 32, 0), v(n * 32, 0), vf(n, 0);
  for (size_t i = 0; i < n; ++i) {
    std::memcpy(&r[i * 32], &s.sig[i * 65], 32);
    std::memcpy(&sv[i * 32], &s.sig[i * 65 + 32], 32);
    const uint64_t vv = s.sig[i * 65 + 64] + 35 + 2 * CHAIN;
    for (int k = 0; k < 8; ++k) v[i * 32 + 31 - k] = uint8_t(vv >> (8 * k));
  }
  CHECK(eges_sender_batch(sighash.data(), r.data(), sv.data(), v.data(), vf.data(), n, 2, CHAIN, addr.data(),
                          st.data()) == EGES_SUCCESS,
        "sender batch");
  bad = 0;
  for (size_t i = 0; i < n; ++i) bad += st[i] != EGES_OK || std::memcmp(&addr[i * 20], &s.addr[i * 20], 20);
  CHECK(bad == 0, "sender batch: %zu wrong", bad);
}

int main(int argc, char** argv) {
  const int mutations = argc > 1 ? std::atoi(argv[1]) : 20000;
  int ndev = 0;
  g_nodev = hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0;
  const bool trace = std::getenv("SANITIZE_TRACE") != nullptr;
  auto step = [&](const char* s) {
    if (trace) std::fprintf(stderr, "== step %s\n", s), std::fflush(stderr);
  };
  step("keccak");
  keccak_known_answers();
  step("arguments");
  argument_validation();
  step("block structure");
  block_structure(mutations);
  step("init");
  const bool gpu = eges_init(1, 0) == EGES_SUCCESS;
  if (!gpu) {
    std::printf("no GPU engine (%s): host-only paths\n", eges_last_error());
    coalescer_without_device();
  } else {
    argument_validation();
    for (size_t n : {1u, 37u, 1000u, 5000u, 70000u}) batch_recover(n);
    single_item_threads(8, 300);
    signed_block(300);
    // the chunked host-buffer path (a shard of >= 512k items in EGES_HOST_PARTS chunks)
    step("host chunks");
    eges_test_set_knob("EGES_HOST_PARTS", 5);
    batch_recover(600011);
    eges_test_set_knob("EGES_HOST_PARTS", 8);
    block_structure(2000);
    eges_shutdown();
  }
  std::printf("sanitize_host: %ld checks, %ld mismatches (%s)\n", g_checks, g_fail, gpu ? "GPU data paths" : "host only");
  return g_fail ? 1 : 0;
}
