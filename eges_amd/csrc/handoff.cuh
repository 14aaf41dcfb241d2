#pragma once
// Hand-offs between the waves of one workgroup through LDS (the mid-size kernel's roles,
// k_recover_mid.hip, and the latency kernels' split form, k_recover_lat.hip).
//
// A producer publishes a value (a flag 1, or a running count) after its LDS data with a
// workgroup release fence; consumers poll until the value reaches what they need, then acquire.
// Every wait is bounded (~1 s at the shader clock, against microseconds in normal operation): a
// wait that runs out, or that sees another wave of the workgroup give up first, marks the
// workgroup's error word and returns false. The wave that writes the outputs checks that word
// after its last wait (every other wave's last wait precedes a value that wave consumes), and
// then writes ST_ENGINE_FAULT and no address for the workgroup's items: the host-buffer entries
// return EGES_E_HIP for such a call, and EGES_DIAG_HANDOFF counts it. So a logic error can
// neither hang the device nor yield a status-OK result computed from LDS that was never written.
#include "core.cuh"

namespace eges {

DEV uint32_t ho_load(const uint32_t* f) {
  return __hip_atomic_load(const_cast<uint32_t*>(f), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// publish v (after this wave's earlier LDS writes); skip: tests only (KNOB_TEST_SKIP_FLAG)
DEV void ho_set(uint32_t* f, uint32_t v = 1u, bool skip = false) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  if (!skip && (threadIdx.x & 63) == 0) __hip_atomic_store(f, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// wait until *f >= k; false (and *err set) on timeout or when another wave has already failed
template <int SLEEP>
DEV bool ho_wait(const uint32_t* f, uint32_t k, uint32_t* err) {
  constexpr uint32_t POLLS = (1u << 25) / SLEEP;  // x (64 SLEEP + ~20) cycles: ~1 s
#pragma unroll 1
  for (uint32_t it = 0; it < POLLS; ++it) {
    if (ho_load(f) >= k) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
      return true;
    }
    if (ho_load(err) != 0u) break;
    __builtin_amdgcn_s_sleep(SLEEP);
  }
  if ((threadIdx.x & 63) == 0) __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
  return false;
}
// the output wave, after its last wait: did any hand-off of this workgroup fail?
DEV bool ho_failed(const uint32_t* err, const Diag& dg) {
  const bool bad = ho_load(err) != 0u;
  if (bad) diag_bump(dg, EGES_DIAG_HANDOFF);
  return bad;
}
// Host-buffer calls launch before their inputs are in the pinned buffer (hostpath.hip Gate): the
// host copies them while the launch is in flight and stores its progress into the gate word
// (coherent pinned memory) piece by piece, in workgroup order. Workgroup 0's first wave alone
// polls that word (a poller per wave over PCIe slowed a 1,000-workgroup launch 2.4x) and mirrors
// every new value into a device word, until the last piece; every other wave waits there for the
// piece its own workgroup reads (gate_step workgroups per piece), so the first workgroups start
// while the host still copies the last ones' inputs and their reads over the bus are spread out
// instead of all at once. No input line can be cached on the device before its piece is open
// (the launch invalidated the caches, and nothing reads an input before its gate), so no
// system-scope cache invalidation follows. A wait that runs out (4 s; the host opens every piece
// on every path, microseconds after its launch) marks gate[1], and the host fails the call rather
// than return results from stale inputs.
DEV bool seq_before(uint32_t have, uint32_t want) { return (int32_t)(have - want) < 0; }
template <class P>
DEV void gate_wait(const P& prm) {
  if (!prm.gate) return;
  constexpr uint64_t BOUND = 400000000ull;  // s_memrealtime ticks (100 MHz): 4 s
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  const uint32_t want = prm.gate_step ? prm.gate_seq - prm.gate_pieces + blockIdx.x / prm.gate_step + 1u : prm.gate_seq;
  if (blockIdx.x == 0 && threadIdx.x < 64) {
    uint32_t* g = const_cast<uint32_t*>(prm.gate);
    uint32_t last = prm.gate_seq - prm.gate_pieces;  // (no piece open yet)
#pragma unroll 1
    for (;;) {
      const uint32_t v = __builtin_amdgcn_readfirstlane(__hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
      if (v != last && !seq_before(v, last)) {
        if (threadIdx.x == 0) __hip_atomic_store(prm.gate_dev, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last = v;
      }
      if (!seq_before(v, prm.gate_seq)) break;
      if (__builtin_amdgcn_s_memrealtime() - t0 > BOUND) {
        if (threadIdx.x == 0) {
          __hip_atomic_store(g + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          __hip_atomic_store(prm.gate_dev, prm.gate_seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // release the waves
        }
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    return;
  }
#pragma unroll 1
  while (seq_before(__hip_atomic_load(prm.gate_dev, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT), want)) {
    if (__builtin_amdgcn_s_memrealtime() - t0 > BOUND + BOUND / 4) break;  // (workgroup 0 marks the failure)
    __builtin_amdgcn_s_sleep(2);
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}
// Stores into pinned host memory and a later flag: round 6 found (tools/host_one_probe2.py on round
// 5's one-launch form, profiles/r06/host_one_probe2_r06_d.txt) that the host can see a flag word
// before bytes the same workgroup stored earlier, although every wave waited for its stores
// (s_waitcnt vmcnt(0)) and thread 0 released at system scope before the flag: the stale bytes were
// whole 256-byte spans of the outputs written last, a second read microseconds later already saw
// them, and they never appeared when the host waited 20 us after the flag or when each lane first
// loaded back, at system scope, a dword of what it had stored. A load of an address cannot complete
// before the store to the same address has landed, so before a workgroup counts itself done the
// lanes that wrote outputs read back the first and the last dword of every output they stored
// (an item's bytes touch at most two 128-byte lines): out_readback, consumed by out_settle so the
// loads have returned before the barrier. (Streams drained by the kernel-end signal need none of
// this: the command processor's end-of-kernel release waits for the writes' confirmation.)
DEV uint32_t rb_sys(const uint8_t* p) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(reinterpret_cast<uintptr_t>(p) & ~(uintptr_t)3);
  return __hip_atomic_load(const_cast<uint32_t*>(w), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
DEV uint32_t rb_span(const uint8_t* p, size_t len) { return rb_sys(p) ^ rb_sys(p + len - 1); }
// every output of item idx (status, address, key) that a recover kernel stored into pinned memory
template <class P>
DEV uint32_t out_readback(const P& prm, uint32_t idx) {
  uint32_t acc = rb_sys(prm.status + idx);
  if (prm.addr) acc ^= rb_span(prm.addr + (size_t)idx * prm.addr_stride, 20);
  if (prm.pub) acc ^= rb_span(prm.pub + (size_t)idx * 65, 65);
  return acc;
}
DEV void out_settle(uint32_t acc) { asm volatile("" ::"v"(acc)); }  // (the loads' values are used: they have returned)

// A gated call's completion (hostpath.hip run_host_shard): after its last output each workgroup
// counts itself done (system-scope release first); the last one stores the call's sequence into
// gate[2], which the host polls instead of synchronising the stream (the kernel-end signal's
// path measured ~5 us from the kernel's end to the sync's return). At kernel level, after the
// body: every wave of the workgroup reaches the barrier. The mid-size kernels only: on the
// latency kernels' 1,000-workgroup grids the per-workgroup system-scope release cost more than
// it saved (C3 0.184-0.188 -> 0.201-0.207 ms, profiles/r04/gate_r04_q.txt).
template <class P>
DEV void gate_done(const P& prm) {
  if (!prm.gate || !prm.gate_word) return;
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    const uint32_t c = __hip_atomic_fetch_add(prm.gate_dev + 1, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (c == gridDim.x - 1) {
      __hip_atomic_store(prm.gate_dev + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(const_cast<uint32_t*>(prm.gate) + 2, prm.gate_seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}
// tests only: workgroup 0's producer of flag k skips publishing it once per launch
template <class P>
DEV bool ho_skip(const P& prm, int k) {
  return prm.test_skip_flag == (uint32_t)k + 1u && blockIdx.x == prm.test_skip_block;
}

}  // namespace eges
