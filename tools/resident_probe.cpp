// Round trip of a small job to a GPU: a launch of an empty one-workgroup kernel + stream sync,
// against a resident workgroup that polls a job word in coherent pinned host memory and answers
// in it (the latency a resident single-call server would pay instead). Bounded: the resident
// kernel exits on a stop word, after STOP_POLLS idle polls, or after its job count. One JSON line.
//   build: hipcc --offload-arch=gfx950 -O2 -std=c++17 tools/resident_probe.cpp -o tools/resident_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <vector>

using clk = std::chrono::steady_clock;

__global__ void empty_kernel(uint32_t* out) {
  if (threadIdx.x == 0) out[0] = 1u;
}

// ctl[0]: job sequence (host), ctl[1]: done sequence (GPU), ctl[2]: stop (host), ctl[3]: payload
__global__ void resident_kernel(uint32_t* ctl, uint32_t max_jobs, uint32_t idle_polls) {
  uint32_t seen = 0, idle = 0;
  while (seen < max_jobs && idle < idle_polls) {
    const uint32_t seq = __hip_atomic_load(&ctl[0], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
    if (__hip_atomic_load(&ctl[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u) break;
    if (seq != seen) {
      seen = seq;
      idle = 0;
      if (threadIdx.x == 0) {
        ctl[3] = ctl[3] + 1u;  // the "result"
        __hip_atomic_store(&ctl[1], seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    } else {
      ++idle;
      __builtin_amdgcn_s_sleep(2);
    }
  }
}

int main() {
  const int N = 2000;
  uint32_t* dout;
  if (hipMalloc(&dout, 256)) return 1;
  hipStream_t st;
  (void)hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
  std::vector<double> a, b;
  for (int i = 0; i < N + 50; ++i) {
    const auto t0 = clk::now();
    hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, st, dout);
    (void)hipStreamSynchronize(st);
    if (i >= 50) a.push_back(std::chrono::duration<double, std::micro>(clk::now() - t0).count());
  }
  uint32_t* ctl;
  if (hipHostMalloc(&ctl, 4096, hipHostMallocCoherent)) return 2;
  for (int i = 0; i < 16; ++i) ctl[i] = 0;
  hipStream_t sr;
  (void)hipStreamCreateWithFlags(&sr, hipStreamNonBlocking);
  // at most N + 50 jobs; exits after ~4M idle polls (seconds) if the host stops answering
  hipLaunchKernelGGL(resident_kernel, dim3(1), dim3(64), 0, sr, ctl, (uint32_t)(N + 50), 4u << 20);
  volatile uint32_t* v = ctl;
  bool ok = true;
  for (int i = 1; i <= N + 50 && ok; ++i) {
    const auto t0 = clk::now();
    std::atomic_thread_fence(std::memory_order_release);
    v[0] = (uint32_t)i;
    while (v[1] != (uint32_t)i) {
      if (std::chrono::duration<double>(clk::now() - t0).count() > 1.0) {
        ok = false;
        break;
      }
    }
    if (i > 50) b.push_back(std::chrono::duration<double, std::micro>(clk::now() - t0).count());
  }
  v[2] = 1u;
  (void)hipStreamSynchronize(sr);
  auto med = [](std::vector<double> x) {
    std::sort(x.begin(), x.end());
    return x.empty() ? 0.0 : x[x.size() / 2];
  };
  auto p99 = [](std::vector<double> x) {
    std::sort(x.begin(), x.end());
    return x.empty() ? 0.0 : x[x.size() * 99 / 100];
  };
  std::printf("{\"metric\": \"small-job round trip, us\", \"launch_sync_p50\": %.2f, \"launch_sync_p99\": %.2f, "
              "\"resident_p50\": %.2f, \"resident_p99\": %.2f, \"jobs\": %d, \"ok\": %s, \"payload\": %u}\n",
              med(a), p99(a), med(b), p99(b), N, ok ? "true" : "false", ctl[3]);
  return ok ? 0 : 3;
}
