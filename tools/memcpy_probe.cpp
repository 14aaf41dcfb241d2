// Host <-> device copy rates on the GPU box, for the host-buffer pipeline (capi.hip
// run_host_shard): host memcpy from pageable into pinned memory (1 and 4 threads), DMA from pinned
// memory, pageable hipMemcpy (HIP's own staging), and the price of hipHostRegister.
//   build: hipcc --offload-arch=gfx950 -O2 -std=c++17 tools/memcpy_probe.cpp -o tools/memcpy_probe -lpthread
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

using clk = std::chrono::steady_clock;
static double ms_since(clk::time_point t0) { return std::chrono::duration<double, std::milli>(clk::now() - t0).count(); }

int main() {
  const size_t B = size_t(25) << 20;  // one 256k-signature chunk of msg + sig is ~25 MB
  std::vector<uint8_t> src(B), dst(B);
  for (size_t i = 0; i < B; ++i) src[i] = (uint8_t)(i * 131u);
  uint8_t *pin, *dev;
  if (hipHostMalloc(&pin, B, hipHostMallocDefault) || hipMalloc(&dev, B)) return 1;
  hipStream_t st;
  (void)hipStreamCreate(&st);
  auto rate = [&](const char* what, int reps, auto fn) {
    fn();
    double best = 1e30;
    for (int r = 0; r < reps; ++r) {
      const auto t0 = clk::now();
      fn();
      best = std::min(best, ms_since(t0));
    }
    std::printf("%-44s %8.3f ms  %7.1f GB/s\n", what, best, B / best / 1e6);
  };
  rate("memcpy pageable -> pinned, 1 thread", 5, [&] { std::memcpy(pin, src.data(), B); });
  for (int T : {2, 4, 8}) {
    char name[64];
    std::snprintf(name, sizeof name, "memcpy pageable -> pinned, %d threads", T);
    rate(name, 5, [&] {
      std::vector<std::thread> th;
      for (int t = 0; t < T; ++t)
        th.emplace_back([&, t] {
          const size_t lo = B * t / T, hi = B * (t + 1) / T;
          std::memcpy(pin + lo, src.data() + lo, hi - lo);
        });
      for (auto& x : th) x.join();
    });
  }
  rate("hipMemcpyAsync pinned -> device (DMA)", 5, [&] {
    (void)hipMemcpyAsync(dev, pin, B, hipMemcpyHostToDevice, st);
    (void)hipStreamSynchronize(st);
  });
  rate("hipMemcpyAsync device -> pinned (DMA)", 5, [&] {
    (void)hipMemcpyAsync(pin, dev, B, hipMemcpyDeviceToHost, st);
    (void)hipStreamSynchronize(st);
  });
  rate("hipMemcpyAsync pageable -> device", 5, [&] {
    (void)hipMemcpyAsync(dev, src.data(), B, hipMemcpyHostToDevice, st);
    (void)hipStreamSynchronize(st);
  });
  rate("hipMemcpyAsync device -> pageable", 5, [&] {
    (void)hipMemcpyAsync(dst.data(), dev, B, hipMemcpyDeviceToHost, st);
    (void)hipStreamSynchronize(st);
  });
  {
    std::vector<uint8_t> big(size_t(101) << 20, 1);
    const auto t0 = clk::now();
    const hipError_t e = hipHostRegister(big.data(), big.size(), hipHostRegisterDefault);
    const double reg = ms_since(t0);
    const auto t1 = clk::now();
    if (e == hipSuccess) (void)hipHostUnregister(big.data());
    std::printf("hipHostRegister 101 MB: %.3f ms (rc %d), unregister %.3f ms\n", reg, (int)e, ms_since(t1));
  }
  return 0;
}
