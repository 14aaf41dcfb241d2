// Native-thread benchmark of the single-item C-ABI entries (eges_ecdsa_recover, the call a Go
// caller makes per crypto.Ecrecover, and eges_ecdsa_verify per crypto.VerifySignature;
// INTEGRATION.md §2): one-caller latencies, then T threads x M recover calls, every result
// checked against the synthetic signer's address. Prints one JSON line.
//   build: hipcc --offload-arch=gfx950 -O2 -std=c++17 tools/single_bench.cpp -Iinclude
//          -Leges_amd -leges -Wl,-rpath,'$ORIGIN/../eges_amd' -o tools/single_bench
//   run:   tools/single_bench [threads=8] [calls=2000]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "eges.h"

int main(int argc, char** argv) {
  const int T = argc > 1 ? std::atoi(argv[1]) : 8;
  const int M = argc > 2 ? std::atoi(argv[2]) : 2000;
  const size_t n = 4096;
  if (eges_init(1, 0) != EGES_SUCCESS) {
    std::fprintf(stderr, "init: %s\n", eges_last_error());
    return 1;
  }
  uint8_t *dm, *ds, *da;
  if (hipMalloc(&dm, n * 32) || hipMalloc(&ds, n * 65) || hipMalloc(&da, n * 20)) return 1;
  if (eges_synth_sign_dev(0, 555000, n, dm, ds, da, nullptr) != EGES_SUCCESS) return 1;
  std::vector<uint8_t> msg(n * 32), sig(n * 65), addr(n * 20);
  if (hipDeviceSynchronize() || hipMemcpy(msg.data(), dm, n * 32, hipMemcpyDeviceToHost) ||
      hipMemcpy(sig.data(), ds, n * 65, hipMemcpyDeviceToHost) ||
      hipMemcpy(addr.data(), da, n * 20, hipMemcpyDeviceToHost))
    return 1;
  std::atomic<long> bad{0};
  auto one = [&](size_t i) {
    uint8_t pub[65];
    if (eges_ecdsa_recover(pub, &sig[i * 65], &msg[i * 32]) != 1) {
      ++bad;
      return;
    }
    uint8_t a[32];
    eges_keccak256(pub + 1, 64, a);
    if (std::memcmp(a + 12, &addr[i * 20], 20) != 0) ++bad;
  };
  using clk = std::chrono::steady_clock;
  // one caller: per-call latency
  std::vector<double> lat;
  for (int k = 0; k < 300; ++k) {
    const auto t0 = clk::now();
    one((size_t)k % n);
    lat.push_back(std::chrono::duration<double, std::milli>(clk::now() - t0).count());
  }
  std::sort(lat.begin() + 20, lat.end());
  const double p50 = lat[20 + (lat.size() - 20) / 2], p99 = lat[20 + (lat.size() - 20) * 99 / 100];
  // one caller: eges_ecdsa_verify (crypto.VerifySignature's seam) against the recovered keys
  std::vector<double> vlat;
  for (int k = 0; k < 300; ++k) {
    const size_t i = (size_t)k % n;
    uint8_t pub[65];
    if (eges_ecdsa_recover(pub, &sig[i * 65], &msg[i * 32]) != 1) ++bad;
    const auto t0 = clk::now();
    if (eges_ecdsa_verify(&sig[i * 65], &msg[i * 32], pub, 65) != 1) ++bad;
    vlat.push_back(std::chrono::duration<double, std::milli>(clk::now() - t0).count());
  }
  std::sort(vlat.begin() + 20, vlat.end());
  const double vp50 = vlat[20 + (vlat.size() - 20) / 2];
  // T callers
  std::vector<std::thread> th;
  const auto t0 = clk::now();
  for (int t = 0; t < T; ++t)
    th.emplace_back([&, t] {
      for (int k = 0; k < M; ++k) one((size_t)(t * 7919 + k * 31) % n);
    });
  for (auto& x : th) x.join();
  const double dt = std::chrono::duration<double>(clk::now() - t0).count();
  std::printf("{\"metric\": \"single-item eges_ecdsa_recover\", \"p50_ms_one_caller\": %.4f, \"p99_ms_one_caller\": %.4f, "
              "\"verify_p50_ms_one_caller\": %.4f, \"threads\": %d, \"calls_per_thread\": %d, \"recoveries_per_s\": %.1f, "
              "\"errors\": %ld}\n",
              p50, p99, vp50, T, M, (double)T * M / dt, bad.load());
  eges_shutdown();
  return bad.load() ? 2 : 0;
}
