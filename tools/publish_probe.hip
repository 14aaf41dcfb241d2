// Publication probe (round 6): can the host see a word that a kernel stored
// into pinned host memory AFTER its earlier output stores (fence + flag) before it sees those
// outputs? The round-5 one-launch host form (profiles/r05/removed_host_one_r05.diff) read stale
// outputs after a block's done word; this probe repeats the publication with a kernel that does
// nothing else, so no compute path (redo passes, batched inversions, slot loops) is involved.
//
// Each call: `blocks` workgroups of 256 threads; block b first spins b * gap_us (so the blocks
// finish one after another and the host is already waiting at each flag), then every thread
// writes its K items (idx = k * GT + g, k = 0 .. K-1, like the lane-serial kernel's phase E):
// five dwords of "address" (20 B per item) and one status byte, values a function of (call, idx).
// Publication modes:
//   block : each block, after `s_waitcnt vmcnt(0)` + barrier + system-scope release fence, stores
//           the call id into done[b] (the one-launch form); the host copies block b's items as
//           soon as done[b] flips
//   last  : each block: barrier + system release + agent-scope counter; the last block stores the
//           call id into one completion word with a system-scope release (handoff.cuh gate_done,
//           and the resident server's done word); the host copies everything when it flips
//   sync  : no flag; the host copies after hipStreamSynchronize (the kernel-end signal)
// Output memory: default (hipHostMallocDefault) | coherent | noncoherent. The flag words are
// always coherent. Optional host delay (us) between seeing a flag and reading the outputs.
// After each call's stream sync the host re-reads the pinned outputs: every byte must then be
// the call's own (it always was, in round 5); a copy that differs from the expected bytes is a
// stale read. Reports per configuration: calls, stale items, stale 256-byte regions, their
// offsets modulo 256 / 64, the slot k and block of each stale item.
//
// Load (optional 8th argument): while the probe kernel runs, a second kernel on another stream
// keeps the memory system busy until the probe's last block is due: 1 device memory (16-B loads
// and stores over a 1 GiB buffer), 2 reads of pinned host memory, 3 writes to pinned host memory,
// 4 = 1 + 2 + 3 (the round-5 one-launch kernel read its inputs from and wrote its outputs to
// pinned memory while every other CU streamed its L2-missing workspace).
//
// Build: hipcc --offload-arch=gfx950 -O2 -std=c++17 tools/publish_probe.hip -o tools/publish_probe
// Run:   tools/publish_probe <mode> <mem> <calls> <blocks> <gap_us> <delay_us> [K] [load]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#define CK(x)                                                                           \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) {                                                             \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(2);                                                                          \
    }                                                                                   \
  } while (0)

constexpr int WG = 256;

__host__ __device__ inline uint32_t val(uint32_t call, uint32_t idx, uint32_t i) {
  uint32_t x = call * 0x9E3779B1u ^ (idx * 0x85EBCA77u + i * 0xC2B2AE3Du);
  x ^= x >> 15;
  x *= 0x2C1B3C6Du;
  x ^= x >> 12;
  return x;
}

struct Prm {
  uint8_t* status;
  uint8_t* addr;
  uint32_t* done;     // coherent: per-block words (block) or [0] completion, (last)
  uint32_t* counter;  // device memory (last)
  uint32_t call, n, K, mode;  // mode 0 block, 1 last, 2 sync
  uint64_t gap_ticks;
};

__global__ void __launch_bounds__(WG) probe_kernel(Prm p) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  const uint64_t until = t0 + (uint64_t)blockIdx.x * p.gap_ticks;
  while (__builtin_amdgcn_s_memrealtime() < until) __builtin_amdgcn_s_sleep(2);
  const uint32_t GT = gridDim.x * WG, g = blockIdx.x * WG + threadIdx.x;
  for (uint32_t k = 0; k < p.K; ++k) {
    const uint32_t idx = k * GT + g;
    if (idx >= p.n) break;
    p.status[idx] = (uint8_t)(p.call & 0xff);
    uint32_t* dst = reinterpret_cast<uint32_t*>(p.addr + (size_t)idx * 20);
#pragma unroll
    for (int i = 0; i < 5; ++i) dst[i] = val(p.call, idx, i);
  }
  if (p.mode == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      __hip_atomic_store(p.done + blockIdx.x, p.call, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  } else if (p.mode == 1) {
    __syncthreads();
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      const uint32_t c = __hip_atomic_fetch_add(p.counter, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
      if (c == gridDim.x - 1) {
        __hip_atomic_store(p.counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(p.done, p.call, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
  }
}

// the load kernel: until s_memrealtime passes `until`, each thread streams 16-B words
__global__ void __launch_bounds__(WG) load_kernel(uint4* dev, size_t dev_words, uint4* hin, uint4* hout, size_t host_words,
                                                  uint32_t kinds, uint64_t ticks) {
  const uint64_t until = __builtin_amdgcn_s_memrealtime() + ticks;
  const size_t tid = (size_t)blockIdx.x * WG + threadIdx.x, nt = (size_t)gridDim.x * WG;
  uint4 acc = make_uint4(0, 0, 0, 0);
  size_t i = tid, j = tid;
  while (__builtin_amdgcn_s_memrealtime() < until) {
#pragma unroll 1
    for (int r = 0; r < 16; ++r) {
      if (kinds & 1u) {
        const uint4 v = dev[i];
        acc.x ^= v.x;
        acc.y += v.y;
        dev[(i + dev_words / 2) % dev_words] = make_uint4(v.x + 1u, v.y, v.z ^ acc.x, v.w);
        i = (i + nt * 7) % dev_words;
      }
      if (kinds & 2u) {
        const uint4 v = hin[j];
        acc.z ^= v.z;
        acc.w += v.w;
      }
      if (kinds & 4u) hout[j] = make_uint4(acc.x, (uint32_t)j, acc.z, acc.w);
      j = (j + nt) % host_words;
    }
  }
  if (acc.x == 0x12345678u && acc.y == 0x9abcdefu) dev[0] = acc;  // (keeps the loads)
}

static void spin_us(double us) {
  if (us <= 0) return;
  const auto t0 = std::chrono::steady_clock::now();
  while (std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() < us) {
  }
}

int main(int argc, char** argv) {
  if (argc < 7) {
    fprintf(stderr, "usage: %s block|last|sync default|coherent|noncoherent calls blocks gap_us delay_us [K]\n", argv[0]);
    return 2;
  }
  const std::string mode_s = argv[1], mem_s = argv[2];
  const int calls = atoi(argv[3]), blocks = atoi(argv[4]);
  const double gap_us = atof(argv[5]), delay_us = atof(argv[6]);
  const uint32_t K = argc > 7 ? (uint32_t)atoi(argv[7]) : 4u;
  const int load = argc > 8 ? atoi(argv[8]) : 0;
  const uint32_t kinds = load == 4 ? 7u : load == 1 ? 1u : load == 2 ? 2u : load == 3 ? 4u : 0u;
  const uint32_t mode = mode_s == "block" ? 0u : mode_s == "last" ? 1u : 2u;
  const unsigned flags = mem_s == "coherent" ? hipHostMallocCoherent
                         : mem_s == "noncoherent" ? hipHostMallocNonCoherent
                                                  : hipHostMallocDefault;
  const uint32_t GT = (uint32_t)blocks * WG, n = GT * K;
  CK(hipSetDevice(0));
  uint8_t *status, *addr;
  uint32_t *done, *counter;
  CK(hipHostMalloc(reinterpret_cast<void**>(&status), n, flags));
  CK(hipHostMalloc(reinterpret_cast<void**>(&addr), (size_t)n * 20, flags));
  CK(hipHostMalloc(reinterpret_cast<void**>(&done), (size_t)blocks * 4 + 64, hipHostMallocCoherent));
  CK(hipMalloc(&counter, 64));
  CK(hipMemset(counter, 0, 64));
  unsigned got = 0;
  CK(hipHostGetFlags(&got, addr));
  std::memset(status, 0, n);
  std::memset(addr, 0, (size_t)n * 20);
  std::memset(done, 0, (size_t)blocks * 4 + 64);
  hipStream_t st, sl;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&sl, hipStreamNonBlocking));
  uint4 *ldev = nullptr, *lhin = nullptr, *lhout = nullptr;
  const size_t dev_words = (size_t(1) << 30) / 16, host_words = (size_t(64) << 20) / 16;
  if (kinds) {
    CK(hipMalloc(&ldev, dev_words * 16));
    CK(hipMemset(ldev, 1, dev_words * 16));
    CK(hipHostMalloc(reinterpret_cast<void**>(&lhin), host_words * 16, hipHostMallocDefault));
    CK(hipHostMalloc(reinterpret_cast<void**>(&lhout), host_words * 16, hipHostMallocDefault));
    std::memset(lhin, 3, host_words * 16);
  }
  std::vector<uint8_t> cst(n), cad((size_t)n * 20);
  Prm p{status, addr, done, counter, 0, n, K, mode, (uint64_t)(gap_us * 100.0)};  // s_memrealtime: 100 MHz
  long stale_items = 0, stale_regions = 0, after_sync_bad = 0, stale_calls = 0, status_stale = 0;
  std::map<int, long> off256, off64, slot_hist, len_hist;
  std::vector<long> blocks_hit;
  double flag_wait_us = 0;
  const auto T0 = std::chrono::steady_clock::now();
  for (int c = 0; c < calls; ++c) {
    p.call = 0x1000u + (uint32_t)c * 7u + 1u;
    hipLaunchKernelGGL(probe_kernel, dim3(blocks), dim3(WG), 0, st, p);
    CK(hipGetLastError());
    if (kinds) {  // after the probe's blocks are placed: the load takes the remaining slots
      hipLaunchKernelGGL(load_kernel, dim3(2048), dim3(WG), 0, sl, ldev, dev_words, lhin, lhout, host_words, kinds,
                         (uint64_t)((blocks * gap_us + 200.0) * 100.0));
      CK(hipGetLastError());
    }
    auto copy_block = [&](uint32_t b) {
      for (uint32_t k = 0; k < K; ++k) {
        const size_t lo = (size_t)k * GT + (size_t)b * WG;
        std::memcpy(cst.data() + lo, status + lo, WG);
        std::memcpy(cad.data() + lo * 20, addr + lo * 20, (size_t)WG * 20);
      }
    };
    if (mode == 0) {
      for (int b = 0; b < blocks; ++b) {
        const auto w0 = std::chrono::steady_clock::now();
        while (__atomic_load_n(done + b, __ATOMIC_ACQUIRE) != p.call) __builtin_ia32_pause();
        flag_wait_us += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - w0).count();
        spin_us(delay_us);
        copy_block((uint32_t)b);
      }
    } else if (mode == 1) {
      while (__atomic_load_n(done, __ATOMIC_ACQUIRE) != p.call) __builtin_ia32_pause();
      spin_us(delay_us);
      for (int b = 0; b < blocks; ++b) copy_block((uint32_t)b);
    }
    CK(hipStreamSynchronize(st));
    if (kinds) CK(hipStreamSynchronize(sl));
    if (mode == 2)
      for (int b = 0; b < blocks; ++b) copy_block((uint32_t)b);
    bool any = false;
    long run_end = -1;  // byte offset one past the last stale byte seen (merges a region's items)
    for (uint32_t idx = 0; idx < n; ++idx) {
      bool bad = cst[idx] != (uint8_t)(p.call & 0xff);
      if (bad) ++status_stale;
      bool abad = false;
      for (int i = 0; i < 5 && !abad; ++i) {
        uint32_t v;
        std::memcpy(&v, cad.data() + (size_t)idx * 20 + 4 * i, 4);
        abad = v != val(p.call, idx, (uint32_t)i);
      }
      for (int i = 0; i < 5; ++i) {
        uint32_t v;
        std::memcpy(&v, addr + (size_t)idx * 20 + 4 * i, 4);
        if (v != val(p.call, idx, (uint32_t)i)) {
          ++after_sync_bad;
          break;
        }
      }
      if (!abad) continue;
      any = true;
      ++stale_items;
      const uint32_t k = idx / GT, b = (idx % GT) / WG;
      ++slot_hist[(int)k];
      if ((long)idx * 20 >= run_end) {  // a new stale region: find its exact byte extent
        long s = (long)idx * 20, e = s;
        const long lim = (long)n * 20;
        auto byte_bad = [&](long o) {
          const uint32_t it = (uint32_t)(o / 20), i = (uint32_t)((o % 20) / 4);
          uint32_t v;
          std::memcpy(&v, cad.data() + (size_t)it * 20 + 4 * i, 4);
          const uint32_t w = val(p.call, it, i);
          return ((v >> (8 * (o % 4))) & 0xff) != ((w >> (8 * (o % 4))) & 0xff);
        };
        while (s > 0 && byte_bad(s - 1)) --s;
        while (e < lim && byte_bad(e)) ++e;
        // first / last differing byte (a byte that happens to match both values is fine)
        ++stale_regions;
        ++off256[(int)(s % 256)];
        ++off64[(int)(s % 64)];
        ++len_hist[(int)(e - s)];
        blocks_hit.push_back((long)b);
        run_end = e;
      }
    }
    if (any) ++stale_calls;
  }
  const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - T0).count();
  printf("{\"mode\": \"%s\", \"mem\": \"%s\", \"host_flags\": %u, \"calls\": %d, \"blocks\": %d, \"K\": %u, \"gap_us\": %.2f, "
         "\"delay_us\": %.2f, \"load\": %d, \"stale_calls\": %ld, \"stale_items\": %ld, \"stale_regions\": %ld, \"status_stale\": %ld, "
         "\"after_sync_bad\": %ld, \"mean_flag_wait_us\": %.2f, \"secs\": %.2f",
         mode_s.c_str(), mem_s.c_str(), got, calls, blocks, K, gap_us, delay_us, load, stale_calls, stale_items, stale_regions,
         status_stale, after_sync_bad, mode == 0 ? flag_wait_us / ((double)calls * blocks) : 0.0, secs);
  auto dump = [](const char* name, const std::map<int, long>& m) {
    printf(", \"%s\": {", name);
    bool first = true;
    for (auto& kv : m) {
      printf("%s\"%d\": %ld", first ? "" : ", ", kv.first, kv.second);
      first = false;
    }
    printf("}");
  };
  dump("region_start_mod256", off256);
  dump("region_start_mod64", off64);
  dump("region_bytes", len_hist);
  dump("slot_k", slot_hist);
  printf(", \"blocks_hit\": [");
  for (size_t i = 0; i < blocks_hit.size() && i < 40; ++i) printf("%s%ld", i ? ", " : "", blocks_hit[i]);
  printf("]}\n");
  return 0;
}
