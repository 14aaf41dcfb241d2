// Internal interface between the host engine (engine.h, capi.hip) and the kernels (k_*.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "knobs.h"

namespace eges {

// Record layout produced by the prep kernels: 25 SoA rows of n_pad words
// (z[8], r[8], s[8], meta) — see kernels.hip.
constexpr int REC_ROWS = 25;
// vflags bit set by tx_rows_kernel when the wire-format transaction failed to decode
// (the public EGES_VF_* bits are 1, 2, 4: include/eges.h)
constexpr uint8_t VF_DECODE_ERR = 0x8;
// The recover kernel keeps per-signature state between its phases in SLOT_ROWS uint4 rows of
// n_pad entries right after the record rows (k_recover.hip). A thread owns <= MAX_SLOTS.
constexpr int SLOT_ROWS = 12;
constexpr uint32_t MAX_SLOTS = 32;
// Signatures per device pass of the batch entries (bounds the per-call scratch memory).
constexpr size_t PASS_MAX = size_t(1) << 21;
inline size_t recover_scratch_bytes(size_t n_pad) { return n_pad * ((size_t)REC_ROWS * 4 + (size_t)SLOT_ROWS * 16); }
__host__ __device__ inline uint4* recover_slots(const uint32_t* rec, uint32_t n_pad) {
  return reinterpret_cast<uint4*>(const_cast<uint32_t*>(rec) + (size_t)REC_ROWS * n_pad);
}

struct RecoverParams {
  const uint32_t* rec;
  uint32_t n, n_pad;
  uint8_t* status;
  uint8_t* addr;  // nullable, n*20
  uint8_t* pub;   // nullable, n*65
  const uint32_t* gtab;
  uint32_t* ws;
  uint32_t addr_stride = 20;  // bytes between consecutive addresses (32 for the EVM precompile's word)
  // latency kernel only: parse msg (n*32) / sig (n*65) bytes itself instead of reading rec rows
  // (prep_ecrecover_kernel fused away for small ecrecover calls)
  const uint8_t* raw_msg = nullptr;
  const uint8_t* raw_sig = nullptr;
  // latency kernel only: 0 the narrow form, 1 the split form (four waves per signature),
  // 2 the three-wave form (k_recover_lat.hip FORM_*)
  uint32_t wide = 0;
  // latency kernel, narrow form: leading workgroups that compute R's y lane-serially (one lane
  // per signature) into the slot rows, tagged with this launch's epoch (set by the launcher)
  uint32_t n_helpers = 0, epoch = 0;
  // diagnostic counters of the device (EGES_DIAG_*, bumped by the rare exact branches; nullable)
  uint32_t* diag = nullptr;
  // host-buffer calls (latency and mid-size kernels only): wait for *gate >= gate_seq before
  // reading inputs (handoff.cuh gate_wait); null: the inputs are in place at launch
  const uint32_t* gate = nullptr;
  uint32_t* gate_dev = nullptr;  // its device-memory mirror (workgroup 0 copies the sequence there)
  uint32_t gate_seq = 0;
  // progressive gate (the mid-size kernels): the host opens the inputs in gate_pieces pieces of
  // gate_step workgroups each (the word reaches gate_seq - gate_pieces + p + 1 once piece p is
  // in place); workgroup b waits for its own piece b / gate_step only. gate_step 0: one gate.
  uint32_t gate_step = 0, gate_pieces = 1;
  // tests only (KNOB_FORCE_REDO): run every exact-redo pass as if an accumulator was poisoned
  uint32_t force_redo = 0;
  // tests only (KNOB_TEST_SKIP_FLAG, handoff.cuh): workgroup test_skip_block's producer of hand-off
  // flag test_skip_flag - 1 skips publishing it
  uint32_t test_skip_flag = 0, test_skip_block = 0;
  // tests only (KNOB_TEST_DELAY_X): the bucket form's wave X sleeps before it reads the wire stage
  uint32_t test_delay_x = 0;
  // latency / mid-size kernels: types.Sender rows straight from the caller's SoA rows (n x 32
  // big-endian sighash, r, s, v, 4-byte aligned; vflags n bytes, nullable) instead of record rows:
  // prep_sender_kernel's classification (sender.cuh sender_meta) fused in (sender_parse_*)
  const uint8_t *snd_h = nullptr, *snd_r = nullptr, *snd_s = nullptr, *snd_v = nullptr, *snd_f = nullptr;
  int snd_signer = 0;
  uint64_t snd_chain_id = 0;
  // mid-size bucket form, crypto.VerifySignature mode (launch_verify_mid): the verify inputs
  // (VerifyParams' pub n x 65, publen, msg n x 32, sig n x 64) and its 0/1 output instead
  const uint8_t *v_pub = nullptr, *v_publen = nullptr, *v_msg = nullptr, *v_sig = nullptr;
  uint8_t* v_ok = nullptr;
  uint32_t* v_fault = nullptr;  // as VerifyParams::fault
  // mid-size bucket form only: wire-format transactions instead of record rows (tx_rows_kernel
  // and prep_sender_kernel fused in): item i is wire_raw[wire_off[first + i] - wire_off[0],
  // wire_off[first + i + 1] - wire_off[0]); wire_raw 4-byte aligned. wire_sighash: n x 32 or null.
  const uint8_t* wire_raw = nullptr;
  const uint64_t* wire_off = nullptr;  // item i's offsets at wire_off[wire_first + i (+ 1)]
  uint64_t wire_first = 0;
  int wire_signer = 0;
  uint64_t wire_chain_id = 0;
  uint8_t* wire_sighash = nullptr;
  // latency kernels (the resident server): after item idx's outputs, out_tag[idx] =
  // out_tag_recover(tag_seq, status, pub bytes) (below), which the host checks against the bytes
  // it reads instead of trusting the order in which they arrive
  uint64_t* out_tag = nullptr;
  uint32_t tag_seq = 0;
};

struct VerifyParams {
  const uint8_t* pub;
  const uint8_t* publen;
  const uint8_t* msg;
  const uint8_t* sig;
  uint32_t n;
  uint8_t* ok;
  const uint32_t* gtab;
  uint32_t* ws;
  uint32_t n_pad;
  uint4* slot;        // VERIFY_SLOT_ROWS rows of n_pad
  uint32_t* order;    // n_pad: processing order (compressed keys first)
  uint32_t* counts;   // 2 counters for the order kernel
  uint32_t* diag = nullptr;   // as RecoverParams
  uint32_t force_redo = 0;
  uint32_t test_skip_flag = 0, test_skip_block = 0;
  // a wave hand-off of an item timed out (handoff.cuh): its ok byte is 0 and a kernel stores 1
  // here (system scope: host-buffer calls give a word of coherent pinned memory; nullable)
  uint32_t* fault = nullptr;
  uint64_t* out_tag = nullptr;  // as RecoverParams (out_tag_verify)
  uint32_t tag_seq = 0;
};
// Output tags of the resident server (single.hip resident_job). Stores into pinned host memory can
// reach the host after a later store of the same workgroup (handoff.cuh, round 6), so the server's
// done word does not by itself make the outputs readable: every item also gets a 64-bit tag over
// the job's sequence and the exact output bytes, and the host accepts an item only when the tag it
// reads matches the bytes it reads (a stale tag, stale bytes or a mix of both do not match; it
// reads again until they do). The same function on both sides.
__host__ __device__ inline uint64_t out_tag_mix(uint64_t h, uint32_t w) {
  h = (h ^ w) * 0x9E3779B97F4A7C15ull;
  return h ^ (h >> 29);
}
// status byte, then the 65-byte key as its first byte and 16 big-endian words
__host__ __device__ inline uint64_t out_tag_recover(uint32_t seq, uint32_t status, uint32_t pub0, const uint32_t be[16]) {
  uint64_t h = out_tag_mix(0x6A09E667F3BCC908ull, seq);
  h = out_tag_mix(h, status);
  h = out_tag_mix(h, pub0);
  for (int j = 0; j < 16; ++j) h = out_tag_mix(h, be[j]);
  return out_tag_mix(h, 0x52u);
}
__host__ __device__ inline uint64_t out_tag_verify(uint32_t seq, uint32_t ok, uint32_t fault) {
  uint64_t h = out_tag_mix(0xBB67AE8584CAA73Bull, seq);
  h = out_tag_mix(h, ok);
  h = out_tag_mix(h, fault);
  return out_tag_mix(h, 0x56u);
}
// Verify scratch: slot rows (P affine, prefix product of s), the order, the two counters.
constexpr int VERIFY_SLOT_ROWS = 7;
inline size_t verify_scratch_bytes(size_t n_pad) { return n_pad * ((size_t)VERIFY_SLOT_ROWS * 16 + 4) + 256; }
inline void verify_scratch_bind(VerifyParams& p, uint8_t* scratch, size_t n_pad) {
  p.n_pad = (uint32_t)n_pad;
  p.slot = reinterpret_cast<uint4*>(scratch);
  p.order = reinterpret_cast<uint32_t*>(scratch + n_pad * (size_t)VERIFY_SLOT_ROWS * 16);
  p.counts = p.order + n_pad;
}

struct SynthParams {
  uint64_t first;
  uint32_t n;
  const uint8_t* msg_in;  // nullable: sign these hashes instead of the derived messages
  uint8_t* msg;           // nullable output
  uint8_t* sig;
  uint8_t* addr;
  const uint32_t* gtab;
  uint32_t* ws;
};

hipError_t launch_init_gtab(uint32_t* gtab, hipStream_t st);
hipError_t launch_prep_ecrecover(const uint8_t* msg, const uint8_t* sig, uint32_t n, uint32_t n_pad, uint32_t* rec,
                                 hipStream_t st);
hipError_t launch_prep_sender(const uint8_t* sighash, const uint8_t* r, const uint8_t* s, const uint8_t* v,
                              const uint8_t* vflags, uint32_t n, uint32_t n_pad, int signer, uint64_t chain_id,
                              uint32_t* rec, hipStream_t st);
hipError_t launch_prep_precompile(const uint8_t* input, const uint32_t* inlen, uint32_t n, uint32_t n_pad,
                                  uint32_t* rec, hipStream_t st);
hipError_t launch_tx_rows(const uint8_t* raw, const uint64_t* offsets, uint64_t first, uint32_t n, int signer,
                          uint64_t chain_id, uint8_t* sighash, uint8_t* r, uint8_t* s, uint8_t* v, uint8_t* vflags,
                          hipStream_t st);
#ifdef EGES_PHASE_STAMPS
hipError_t launch_recover_stamped(const RecoverParams& p, int max_blocks, int ws_blocks, hipStream_t st, uint64_t* stamps);
hipError_t launch_recover_lat_stamped(const RecoverParams& p, hipStream_t st, uint64_t* stamps);
hipError_t launch_recover_mid_stamped(const RecoverParams& p, bool bucket, size_t ws_bytes, hipStream_t st,
                                      uint64_t* stamps);
size_t lat_waves(uint32_t n);
#endif
// max_blocks: the resident grid; ws_blocks: blocks the workspace p.ws was allocated for. A
// launch whose grid would exceed ws_blocks is refused (hipErrorInvalidValue), never run.
hipError_t launch_recover(const RecoverParams& p, int max_blocks, int ws_blocks, hipStream_t st);
// Small batches: one signature per 16-lane row, limb-parallel field arithmetic (k_recover_lat.hip).
// Same inputs (prep records) and outputs as launch_recover; no workspace.
hipError_t launch_recover_lat(const RecoverParams& p, hipStream_t st);
// Mid-size batches: 64 signatures per 4-wave workgroup, one role per wave (k_recover_mid.hip).
// bucket: the bucket form (no workspace, one workgroup per CU); else the windowed form, which
// uses p.ws (ceil(n / 64) blocks of mid_ws_bytes_per_block(), refused beyond ws_bytes).
hipError_t launch_recover_mid(const RecoverParams& p, bool bucket, size_t ws_bytes, hipStream_t st);
size_t mid_ws_bytes_per_block();
constexpr uint32_t MID_SIGS_PER_BLOCK = 64;
hipError_t launch_verify(const VerifyParams& p, int max_blocks, int ws_blocks, hipStream_t st);
// VerifySignature on the mid-size kernel's bucket form (64 items per 4-wave workgroup, one per CU
// at most: n <= 64 x CUs; no workspace)
// two: the two-per-CU bucket form (ring in p.ws: ceil(n / 64) blocks of bkt2_ws_bytes_per_block(),
// refused beyond ws_bytes)
hipError_t launch_verify_mid(const VerifyParams& p, bool two, size_t ws_bytes, hipStream_t st);
hipError_t launch_recover_bkt2(const RecoverParams& p, size_t ws_bytes, hipStream_t st);
size_t bkt2_ws_bytes_per_block();
// one item per 128-thread workgroup (k_recover_lat.hip; wide: 192 threads, three partial sums);
// uses pub/publen/msg/sig/n/ok/gtab only
hipError_t launch_verify_lat(const VerifyParams& p, bool wide, hipStream_t st);

// ---- resident single-call server (k_recover_lat.hip lat_resident_kernel; single.hip Resident).
// A few split-form workgroups stay resident and poll a job word in coherent pinned host memory,
// so a coalesced group of eges_ecdsa_recover / eges_ecdsa_verify calls pays no launch, dispatch or
// completion signal (tools/resident_probe.cpp: 4.6 us round trip against 12 us for an empty
// launch + stream sync).
struct ResidentJob {  // coherent pinned host memory, 128 bytes
  uint32_t seq;   // host: the job's sequence number, stored last (release)
  uint32_t n;     // items (<= the server's cap)
  uint32_t kind;  // RESIDENT_RECOVER / RESIDENT_VERIFY
  uint32_t stop;  // host: exit now
  uint32_t done;  // device: the last finished sequence, stored after every output (release)
  uint32_t pad[27];
};
enum { RESIDENT_RECOVER = 0, RESIDENT_VERIFY = 1 };
// the data area (pinned, cap items): recover msg | sig | pub | status; verify pub | publen | msg |
// sig | ok | fault word (offsets from resident_layout)
struct ResidentLayout {
  size_t msg, sig, pub, status;        // recover
  size_t vpub, vpublen, vmsg, vsig, vok, vfault;  // verify
  size_t tag;                                     // cap 64-bit output tags (both kinds)
  size_t total;
};
__host__ __device__ inline ResidentLayout resident_layout(uint32_t cap) {
  ResidentLayout L;
  const size_t c = cap;
  L.msg = 0;
  L.sig = L.msg + c * 32;
  L.pub = L.sig + c * 65;
  L.status = L.pub + c * 65;
  L.vpub = 0;
  L.vpublen = L.vpub + c * 65;
  L.vmsg = L.vpublen + c;
  L.vsig = L.vmsg + c * 32;
  L.vok = L.vsig + c * 64;
  L.vfault = (L.vok + c + 3) / 4 * 4;
  const size_t end = L.status + c > L.vfault + 4 ? L.status + c : L.vfault + 4;
  L.tag = (end + 7) / 8 * 8;
  L.total = L.tag + c * 8;
  return L;
}
// bytes of ResidentParams::counter: the completion counters, then the job mirror
constexpr uint32_t RESIDENT_COUNTER_BYTES = 256;
struct ResidentParams {
  ResidentJob* job;
  uint8_t* data;
  uint32_t cap;
  uint32_t seen0;        // the last sequence finished before this launch
  uint32_t* counter;     // device memory: 2 completion counters (zero at launch), then the job mirror
  uint64_t idle_ticks;   // exit after this long without a job (s_memrealtime, 100 MHz)
  uint32_t inst;         // this launch's id (nonzero): its workgroups' exit mark in the mirror
  const uint32_t* gtab;
  uint32_t* diag;
};
hipError_t launch_lat_resident(const ResidentParams& p, uint32_t wgs, hipStream_t st);
// Blocks the lane-serial kernels may need for a pass of n signatures at a resident grid of
// max_blocks (grid_for_lane_serial: more than resident when n > max_blocks * WG * MAX_SLOTS).
int lane_serial_grid(uint32_t n, int max_blocks);
hipError_t launch_synth(const SynthParams& p, int max_blocks, hipStream_t st);
int occupancy_recover();
int occupancy_verify();
int occupancy_synth();
size_t ws_bytes_per_block();
size_t gtab_bytes();
int threads_per_block();

}  // namespace eges
