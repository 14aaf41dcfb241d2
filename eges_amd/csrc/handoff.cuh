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
// Outputs in pinned host memory are read by the host only after the stream's completion signal
// (the command processor's end-of-kernel release waits for the writes' confirmation). Round 6
// found (tools/host_one_probe2.py on round 5's one-launch form, profiles/r06/) that a flag word a
// workgroup stores after its outputs, even after every wave's s_waitcnt vmcnt(0) and a system-scope
// release, can reach the host before those outputs: the stale bytes were whole 256-byte spans of
// the outputs written last, a second read microseconds later already saw them, and they never
// appeared when the host waited 20 us after the flag or when each lane first loaded back, at system
// scope, a dword of what it had stored. The gated calls' completion word (a flag of that kind) is
// gone (measured slower than the stream's signal once made safe, profiles/r06/
// removed_gate_word_r06.diff); the resident server's done word is backed by per-item output tags
// the host checks (launch.h out_tag_recover / out_tag_verify).
// tests only: workgroup 0's producer of flag k skips publishing it once per launch
template <class P>
DEV bool ho_skip(const P& prm, int k) {
  return prm.test_skip_flag == (uint32_t)k + 1u && blockIdx.x == prm.test_skip_block;
}

}  // namespace eges
