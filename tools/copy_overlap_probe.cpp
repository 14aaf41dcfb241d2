// Host <-> device copies while the lane-serial recover kernel holds the whole GPU (the host-buffer
// pipeline's situation, hostpath.hip run_host_shard / run_host_pipe): hipMemcpyAsync (ROCclr picks a
// blit kernel, which then waits for free CU slots) against hsa_amd_memory_async_copy (the SDMA
// engines). Prints one JSON line.
//   build: hipcc --offload-arch=gfx950 -O2 -std=c++17 tools/copy_overlap_probe.cpp -Iinclude
//          -Leges_amd -leges -lhsa-runtime64 -Wl,-rpath,'$ORIGIN/../eges_amd' -o tools/copy_overlap_probe
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

#include "eges.h"

using clk = std::chrono::steady_clock;
static double ms_since(clk::time_point t0) { return std::chrono::duration<double, std::milli>(clk::now() - t0).count(); }

static hsa_agent_t g_gpu{0}, g_cpu{0};
static uint32_t g_bdf = 0;

static hsa_status_t pick_agent(hsa_agent_t a, void*) {
  hsa_device_type_t t;
  hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
  if (t == HSA_DEVICE_TYPE_CPU && !g_cpu.handle) g_cpu = a;
  if (t == HSA_DEVICE_TYPE_GPU) {
    uint32_t bdf = 0;
    hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_BDFID, &bdf);
    if (bdf == g_bdf) g_gpu = a;
  }
  return HSA_STATUS_SUCCESS;
}

int main() {
  const size_t n = size_t(1) << 20;
  const size_t B = size_t(25) << 20;  // one 256k-signature chunk of msg + sig
  if (eges_init(1, 0) != EGES_SUCCESS) return 1;
  int bus = 0, dev = 0, fn = 0;
  hipDeviceGetAttribute(&bus, hipDeviceAttributePciBusId, 0);
  hipDeviceGetAttribute(&dev, hipDeviceAttributePciDeviceId, 0);
  g_bdf = (uint32_t)((bus << 8) | (dev << 3) | fn);
  if (hsa_init() != HSA_STATUS_SUCCESS) return 2;
  hsa_iterate_agents(pick_agent, nullptr);
  if (!g_gpu.handle || !g_cpu.handle) {
    std::fprintf(stderr, "no HSA agent for bdf %x\n", g_bdf);
    return 3;
  }
  uint8_t *msg, *sig, *addr, *st, *pin, *dbuf;
  if (hipMalloc(&msg, n * 32) || hipMalloc(&sig, n * 65) || hipMalloc(&addr, n * 20) || hipMalloc(&st, n) ||
      hipMalloc(&dbuf, B) || hipHostMalloc(&pin, B, hipHostMallocDefault))
    return 4;
  std::memset(pin, 7, B);
  std::vector<uint8_t> exp(n * 20);
  if (eges_synth_sign_dev(0, 0, n, msg, sig, addr, nullptr) != EGES_SUCCESS) return 5;
  hipDeviceSynchronize();
  hipStream_t sk, sc;
  hipStreamCreateWithFlags(&sk, hipStreamNonBlocking);
  hipStreamCreateWithFlags(&sc, hipStreamNonBlocking);
  hsa_signal_t sig_done;
  hsa_signal_create(1, 0, nullptr, &sig_done);
  auto hip_copy = [&](bool h2d) {
    const auto t0 = clk::now();
    if (h2d) hipMemcpyAsync(dbuf, pin, B, hipMemcpyHostToDevice, sc);
    else hipMemcpyAsync(pin, dbuf, B, hipMemcpyDeviceToHost, sc);
    hipStreamSynchronize(sc);
    return ms_since(t0);
  };
  auto hsa_copy = [&](bool h2d) {
    const auto t0 = clk::now();
    hsa_signal_store_relaxed(sig_done, 1);
    hsa_status_t s = h2d ? hsa_amd_memory_async_copy(dbuf, g_gpu, pin, g_cpu, B, 0, nullptr, sig_done)
                         : hsa_amd_memory_async_copy(pin, g_cpu, dbuf, g_gpu, B, 0, nullptr, sig_done);
    if (s != HSA_STATUS_SUCCESS) return -1.0;
    hsa_signal_wait_scacquire(sig_done, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_ACTIVE);
    return ms_since(t0);
  };
  auto kernel = [&]() { return eges_ecrecover_batch_dev(0, msg, sig, n, nullptr, addr, st, sk); };
  // idle GPU
  double idle[4] = {1e9, 1e9, 1e9, 1e9};
  for (int r = 0; r < 5; ++r) {
    idle[0] = std::min(idle[0], hip_copy(true));
    idle[1] = std::min(idle[1], hip_copy(false));
    idle[2] = std::min(idle[2], hsa_copy(true));
    idle[3] = std::min(idle[3], hsa_copy(false));
  }
  // under a 1M recover launch (~10 ms): start the kernel, wait 1 ms so its grid is resident, copy
  double busy[4] = {0, 0, 0, 0}, kern = 0;
  const int R = 4;
  for (int w = 0; w < 4; ++w) {
    for (int r = 0; r < R; ++r) {
      hipStreamSynchronize(sk);
      const auto t0 = clk::now();
      if (kernel() != EGES_SUCCESS) return 6;
      while (ms_since(t0) < 1.0) {
      }
      const double c = w == 0 ? hip_copy(true) : w == 1 ? hip_copy(false) : w == 2 ? hsa_copy(true) : hsa_copy(false);
      busy[w] += c / R;
      hipStreamSynchronize(sk);
      kern += ms_since(t0) / (4 * R);
    }
  }
  std::printf(
      "{\"metric\": \"25 MB pinned copy, ms: idle GPU vs under a resident 1M recover launch\", "
      "\"idle\": {\"hip_h2d\": %.3f, \"hip_d2h\": %.3f, \"sdma_h2d\": %.3f, \"sdma_d2h\": %.3f}, "
      "\"under_kernel\": {\"hip_h2d\": %.3f, \"hip_d2h\": %.3f, \"sdma_h2d\": %.3f, \"sdma_d2h\": %.3f}, "
      "\"kernel_call_ms\": %.3f}\n",
      idle[0], idle[1], idle[2], idle[3], busy[0], busy[1], busy[2], busy[3], kern);
  hsa_signal_destroy(sig_done);
  return 0;
}
