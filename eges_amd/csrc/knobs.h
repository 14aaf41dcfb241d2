// Engine knobs and diagnostic counters (host side of libeges.so).
//
// Knobs are read from the environment ONCE, at the first eges_init, and are otherwise changed
// only through eges_test_set_knob (include/eges.h): no call path after init reads the
// environment (getenv racing a host application's setenv is undefined behaviour in glibc).
// The values are atomics, so a test may flip one while other threads run; a call snapshots the
// routing knobs once at its start (engine.h Route), so a change takes effect from the next call.
#pragma once
#include <stdint.h>

namespace eges {

enum KnobId : int {
  KNOB_LAT_MAX = 0,       // batches of at most this many signatures take the latency kernels
  KNOB_LAT_WIDE_MAX,      // latency batches of at most this many take the split (4-wave) form
  KNOB_MID_MAX,           // batches above LAT_MAX and at most this many take the mid-size kernel
  KNOB_MID_FORM,          // mid-size kernel: 1 auto (bucket form while the grid fits one workgroup
                          //   per CU, windowed beyond), 0 windowed form, 2 bucket form
  KNOB_WIRE_FUSED,        // wire-format batches decode inside the recover kernel: 1 latency kernels and
                          //   bucket form, 2 bucket form only, 0 neither
  KNOB_TXROWS_WAVE_MAX,   // wire-format batches of at most this many decode one tx per wave
  KNOB_ROOT_HELPERS,      // 0: the narrow form launches no root-helper workgroups (tests)
  KNOB_OVERLAP,           // device-resident recover batches as S overlapped launches (-1 = auto)
  KNOB_FORCE_REDO,        // tests: run every exact-redo pass as if an accumulator was poisoned
  KNOB_COALESCE_GATHER_US,  // single-item coalescer: a leader's gather window
  KNOB_COALESCE_SPIN_US,    //   a waiting caller spins this long before it blocks
  KNOB_COALESCE_SPINNERS,   //   at most this many callers spin at once
  KNOB_SENDER_FUSED,      // 1: sender rows of latency / mid-size batches are classified inside the
                          //   recover kernel (no prep_sender launch); 0: prep_sender_kernel first
  KNOB_LAT_TRI_MAX,       // latency batches above LAT_WIDE_MAX up to this size: the three-wave form
  KNOB_HOST_PARTS,        // host-buffer shards of >= 2 * PIPE_MIN items without the pipeline: chunks (8;
                          //   at least PIPE_MIN / 2 signatures each)
  KNOB_TEST_SKIP_FLAG,    // tests: k > 0 makes item 0's workgroup's producer of hand-off flag k - 1
                          //   skip publishing it (handoff.cuh), so its consumers time out
  KNOB_TEST_DELAY_X,      // tests: the bucket form's wave X sleeps k x ~3 us before it reads its
                          //   workgroup's wire stage (the stage / part[0] release)
  KNOB_RESIDENT,          // 1: coalesced single calls go to the resident server (single.hip Resident)
  KNOB_RESIDENT_WGS,      //   its workgroups (split form, four waves each)
  KNOB_RESIDENT_CAP,      //   the largest group it takes (larger groups launch on a lane)
  KNOB_RESIDENT_IDLE_US,  //   it exits after this many us without a job (restarted on demand; 500: its workgroups
                          //   leave the CUs to other work soon after a burst of calls, and back-to-back
                          //   callers keep it alive; another process's 1M launch right after a single call
                          //   ran 0.95-1.05 % slower at 1 ms, bench.py secondary.single.resident_tax)
  KNOB_GATE,              // 1: single-chunk host-buffer calls on the mid-size kernels launch first and copy
                          //   their inputs while the launch is in flight (hostpath.hip Gate; the latency
                          //   kernels run ungated)
  KNOB_GATE_STEP,         //   mid-size workgroups per gate piece (8: the host opens the inputs piece by piece
                          //   and each workgroup waits for its own; 0: one piece). C1 0.413-0.415 ->
                          //   0.399-0.400 ms (profiles/r05/gate_step_hostgens_gm_r05_h.txt)
  KNOB_HOST_GENS,         // host-buffer chunks on the lane-serial kernel: resident generations per launch
                          //   (0: the device's EGES_GRID_MULT; fewer generations, more signatures per thread)
  KNOB_VERIFY_MID_GENS,   // VerifySignature batches above LAT_MAX take the bucket form's verify mode while
                          //   its grid is at most this many generations of one workgroup per CU (2: 20k-32k
                          //   items 0.78 -> 0.66-0.67 ms; profiles/r05/formcurve_verify_gens_r05_m.jsonl)
  KNOB_BKT2,              // the bucket form at two workgroups per CU (ring in the workspace, no wire form):
                          //   1 for non-wire recover and verify batches of the mid-size band up to one
                          //   generation at two per CU (n <= 128 x CUs; route.hip mid_bkt2); 2 wherever the
                          //   bucket form runs (tests); 0 never
  KNOB_TEST_RECHECK,      // tests: a host-buffer call whose outputs come back through pinned memory (the
                          //   lanes, the gated mid-size launches, the resident server) re-reads them after the
                          //   work has drained (the stream, or 200 us for the resident server) and fails
                          //   with EGES_E_HIP if any byte differs from what the call returned
  KNOB_COUNT
};

long long knob(KnobId k);

// Diagnostic counters (per device, device memory, incremented by the kernels' rare branches;
// read by eges_diag_counters). Indices are the EGES_DIAG_* values of include/eges.h.
constexpr int DIAG_WORDS = 16;

}  // namespace eges
