// C3 (configs[2]) host-path latency from native code: one Geec block of N EIP-155 transactions
// through eges_sender_batch (host buffers, the call the Go block processor makes through cgo;
// INTEGRATION.md §4), timed around the C call itself (no Python wrapper). Every sender is
// checked against the synthetic signer's address. Linked against libeges_diag.so (EGES_PHASE_STAMPS)
// it also prints the host phase split of the call (hostpath.hip HSTAMP). Prints one JSON line.
//   build: hipcc --offload-arch=gfx950 -O2 -std=c++17 tools/block_bench.cpp -Iinclude
//          -Leges_amd -leges -Wl,-rpath,'$ORIGIN/../eges_amd' -ldl -o tools/block_bench
//   run:   tools/block_bench [txs=1000] [iters=300]
#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "eges.h"

int main(int argc, char** argv) {
  const size_t n = argc > 1 ? (size_t)std::atol(argv[1]) : 1000;
  const int iters = argc > 2 ? std::atoi(argv[2]) : 300;
  const uint64_t chain_id = 930412;  // the Geec chain id (EIP155Signer)
  if (eges_init(1, 0) != EGES_SUCCESS) {
    std::fprintf(stderr, "init: %s\n", eges_last_error());
    return 1;
  }
  // sighash_i = Keccak256("eges-c3" || le64(i)), signed by the synthetic keys on the GPU
  std::vector<uint8_t> h(n * 32), sig(n * 65), exp(n * 20);
  for (size_t i = 0; i < n; ++i) {
    uint8_t in[15] = {'e', 'g', 'e', 's', '-', 'c', '3'};
    for (int k = 0; k < 8; ++k) in[7 + k] = (uint8_t)(i >> (8 * k));
    eges_keccak256(in, sizeof in, &h[i * 32]);
  }
  uint8_t *dh, *ds, *da;
  if (hipMalloc(&dh, n * 32) || hipMalloc(&ds, n * 65) || hipMalloc(&da, n * 20)) return 1;
  if (hipMemcpy(dh, h.data(), n * 32, hipMemcpyHostToDevice)) return 1;
  if (eges_synth_sign_msg_dev(0, 0, n, dh, ds, da, nullptr) != EGES_SUCCESS) return 1;
  if (hipDeviceSynchronize() || hipMemcpy(sig.data(), ds, n * 65, hipMemcpyDeviceToHost) ||
      hipMemcpy(exp.data(), da, n * 20, hipMemcpyDeviceToHost))
    return 1;
  // SoA sender rows: r, s, v = recid + 35 + 2 chain_id, big-endian 32-byte
  std::vector<uint8_t> r(n * 32), s(n * 32), v(n * 32, 0), vf(n, 0), addr(n * 20), st(n);
  for (size_t i = 0; i < n; ++i) {
    std::memcpy(&r[i * 32], &sig[i * 65], 32);
    std::memcpy(&s[i * 32], &sig[i * 65 + 32], 32);
    const uint64_t vv = sig[i * 65 + 64] + 35 + 2 * chain_id;
    for (int k = 0; k < 8; ++k) v[i * 32 + 31 - k] = (uint8_t)(vv >> (8 * k));
  }
  using fn_t = size_t (*)(int64_t*, size_t);
  const fn_t stamps = (fn_t)dlsym(RTLD_DEFAULT, "eges_diag_host_stamps");
  using clk = std::chrono::steady_clock;
  std::vector<double> lat;
  std::vector<double> ph[5];
  long bad = 0;
  for (int it = 0; it < iters + 20; ++it) {
    std::memset(addr.data(), 0, addr.size());
    const auto t0 = clk::now();
    const int rc = eges_sender_batch(h.data(), r.data(), s.data(), v.data(), vf.data(), n, EGES_SIGNER_EIP155, chain_id,
                                     addr.data(), st.data());
    const double ms = std::chrono::duration<double, std::milli>(clk::now() - t0).count();
    if (rc != EGES_SUCCESS || std::memcmp(addr.data(), exp.data(), n * 20) != 0) ++bad;
    for (size_t i = 0; i < n; ++i) bad += st[i] != 0;
    if (it < 20) continue;
    lat.push_back(ms);
    if (stamps) {
      int64_t t[6];
      stamps(t, 6);
      for (int k = 0; k < 5; ++k) ph[k].push_back((t[k + 1] - t[k]) / 1e3);
    }
  }
  auto med = [](std::vector<double> x) {
    std::sort(x.begin(), x.end());
    return x.empty() ? 0.0 : x[x.size() / 2];
  };
  std::vector<double> sl = lat;
  std::sort(sl.begin(), sl.end());
  std::printf("{\"metric\": \"C3 block via eges_sender_batch, native caller\", \"txs\": %zu, \"iters\": %d, "
              "\"median_ms\": %.4f, \"p99_ms\": %.4f, \"errors\": %ld",
              n, iters, sl[sl.size() / 2], sl[sl.size() * 99 / 100], bad);
  if (stamps)
    std::printf(", \"host_phases_us_median\": {\"acquire\": %.2f, \"pack\": %.2f, \"launch\": %.2f, \"sync\": %.2f, "
                "\"unpack\": %.2f}",
                med(ph[0]), med(ph[1]), med(ph[2]), med(ph[3]), med(ph[4]));
  std::printf("}\n");
  eges_shutdown();
  return bad ? 2 : 0;
}
