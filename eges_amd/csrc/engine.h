// Internal interface of the host engine (libeges.so's host side, namespace eges::host): the
// device registry, its per-device resources and knobs (engine.hip), routing and the
// device-resident pipelines (route.hip), the host-buffer paths (hostpath.hip), the single-item
// seam (single.hip); capi.hip holds the C ABI (include/eges.h) over them.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <initializer_list>
#include <memory>
#include <atomic>
#include <mutex>
#include <string>
#include <thread>
#include <type_traits>
#include <vector>

#include "eges.h"
#include "launch.h"

namespace eges::host {

using namespace eges;

constexpr size_t CHUNK = PASS_MAX;  // signatures per device pass (bounds scratch memory)
// host-buffer shards of at least 2 * PIPE_MIN items are split into EGES_HOST_PARTS chunks (copies of
// one chunk overlap the kernels of the previous one; 8 parts at 1M: profiles/r04/c2host_*)
constexpr size_t PIPE_MIN = size_t(1) << 18;
// Single-chunk host-buffer calls whose device region fits this many bytes are staged through
// one pinned host buffer: the caller's inputs are packed on the host, moved by ONE H2D copy,
// and the outputs come back by one D2H copy (a 1000-transaction block otherwise pays five
// pageable H2D and two pageable D2H copies, ~0.1 ms).
constexpr size_t PIN_BYTES = size_t(8) << 20;
#ifndef EGES_PIPE_PARTS
#define EGES_PIPE_PARTS 8
#endif

extern thread_local std::string t_err;

// Publishes a word the GPU polls after this thread's earlier stores into pinned memory. A
// release store is not enough on x86: glibc's memcpy writes large copies with non-temporal
// stores, which TSO does not order before a later store; the sfence drains them first.
inline void publish_u32(uint32_t* w, uint32_t v) {
#if defined(__x86_64__)
  __builtin_ia32_sfence();
#endif
  __atomic_store_n(w, v, __ATOMIC_RELEASE);
}

inline void cpu_relax() {
#if defined(__x86_64__)
  __builtin_ia32_pause();
#else
  std::this_thread::yield();
#endif
}

int set_err(int rc, const char* fmt, ...);
int env_int(const char* name, int dflt);

#define HIPCHK(expr)                                                                                \
  do {                                                                                              \
    hipError_t e_ = (expr);                                                                         \
    if (e_ != hipSuccess) return set_err(EGES_E_HIP, "%s failed: %s", #expr, hipGetErrorString(e_)); \
  } while (0)

// A small-call lane: its own stream, device scratch and pinned staging, so that concurrent
// single-chunk host calls that run on the latency kernel (which needs no shared workspace) do
// not queue behind each other on the device mutex.
constexpr int NLANES = 4;
// A host-buffer call's input gate (handoff.cuh gate_wait): word 0 the last sequence opened, word 1
// set by a wave whose wait ran out. Coherent
// pinned memory, one per device (the gated mid-size calls hold the device mutex).
struct Gate {
  uint32_t* w = nullptr;
  uint32_t* dev = nullptr;  // device word: workgroup 0's mirror of the opened sequence
  uint32_t seq = 0;
};
struct Lane {
  std::mutex mu;
  // the resident server runs on lane 0's stream (its persistent kernel holds that stream's
  // hardware queue): while it does, lane 0 takes no calls
  std::atomic<bool> reserved{false};
  hipStream_t stream = nullptr;
  uint8_t* buf = nullptr;
  size_t buf_cap = 0;
  uint8_t* pin = nullptr;
  uint32_t* vfault = nullptr;  // coherent pinned: a VerifySignature call's hand-off fault word
  hipEvent_t ev_in[2] = {nullptr, nullptr}, ev_k[2] = {nullptr, nullptr};
};

// Resident single-call server of a device (k_recover_lat.hip lat_resident_kernel): a few
// split-form workgroups polling a job word in coherent pinned memory (resident_run below).
struct Resident {
  std::mutex mu;  // one job at a time; a group that finds it busy takes a lane instead
  int lane = 0;
  hipStream_t stream = nullptr;
  ResidentJob* job = nullptr;  // coherent pinned
  uint8_t* data = nullptr;     // pinned, resident_layout (cap)
  uint32_t* counter = nullptr;  // device, 2 words + the job mirror
  uint32_t cap = 0, wgs = 0;
  bool running = false;  // (guarded by mu; while true, the stream's lane is reserved)
  uint32_t seq = 0;  // the last job handed over (== job->done once served)
  uint32_t inst = 0;  // launches so far (each launch's id, nonzero)
  std::chrono::steady_clock::time_point last_use{};
};
struct Dev {
  int id = -1;
  int cus = 0;
  hipStream_t stream = nullptr;
  hipStream_t copy = nullptr;  // host-buffer pipeline: H2D / D2H while `stream` computes
  hipEvent_t last = nullptr;  // completion of the last engine work (workspace users serialise on it)
  hipEvent_t ev_in[2] = {nullptr, nullptr}, ev_k[2] = {nullptr, nullptr};  // per pipeline region
  uint32_t* gtab = nullptr;
  uint32_t* ws = nullptr;
  uint32_t* diag = nullptr;  // DIAG_WORDS counters (eges_diag_counters)
  int mb_recover = 0, mb_verify = 0, mb_synth = 0;
  int gm = 1;  // resident generations of a lane-serial grid (EGES_GRID_MULT)
  int ws_blocks = 0;  // blocks ws (and ws2) hold: every launch's grid is checked against it
  uint8_t* buf = nullptr;  // per-call device scratch, grown on demand
  size_t buf_cap = 0;
  uint8_t* pin = nullptr;  // pinned host staging of single-chunk host-buffer calls (PIN_BYTES)
  Gate gate;               //   and their input gate
  uint32_t* vfault = nullptr;  // coherent pinned: a VerifySignature call's hand-off fault word
  // overlapped recover launches (EGES_OVERLAP): a second stream, workspace and its events
  hipStream_t aux = nullptr;
  uint32_t* ws2 = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  std::mutex mu;
  // device-wide calls in progress (DeviceWide): while nonzero, or while their last enqueued work
  // (`last`) is still pending, the resident server takes no job and is not relaunched
  std::atomic<int> wide{0};
  Lane lanes[NLANES];
  Resident res;
  ~Dev();
};
using DevPtr = std::shared_ptr<Dev>;

// ------------------------------------------------------------------ knobs (knobs.h, engine.hip)
void knobs_load_env();
int knob_index(const char* name);
extern std::atomic<long long> g_knob[KNOB_COUNT];

// The routing knobs of one call, read once at its start (a knob flipped while a call
// runs must not send part of it one way and part another, e.g. a small-lane call onto the
// windowed form's shared workspace).
struct Route {
  size_t lat_max = 0, mid_max = 0;
  uint32_t wide_max = 0, tri_max = 0;
  long long mid_form = 1, wire_fused = 1, overlap = -1, sender_fused = 1, gate = 1, gate_step = 8, bkt2 = 1;
  size_t host_parts = EGES_PIPE_PARTS;
  uint32_t force_redo = 0, skip_flag = 0, delay_x = 0, recheck = 0;
  int host_gens = 0, verify_mid_gens = 1;
  static Route now() {
    Route r;
    r.lat_max = (size_t)std::max<long long>(0, knob(KNOB_LAT_MAX));
    r.mid_max = (size_t)std::max<long long>(0, knob(KNOB_MID_MAX));
    r.wide_max = (uint32_t)std::max<long long>(0, std::min<long long>(knob(KNOB_LAT_WIDE_MAX), 1u << 30));
    r.mid_form = knob(KNOB_MID_FORM);
    r.wire_fused = knob(KNOB_WIRE_FUSED);
    r.overlap = knob(KNOB_OVERLAP);
    r.sender_fused = knob(KNOB_SENDER_FUSED);
    r.gate = knob(KNOB_GATE);
    r.bkt2 = knob(KNOB_BKT2);
    r.gate_step = std::max<long long>(0, std::min<long long>(knob(KNOB_GATE_STEP), 1 << 20));
    r.host_gens = (int)std::max<long long>(0, std::min<long long>(knob(KNOB_HOST_GENS), 8));
    r.verify_mid_gens = (int)std::max<long long>(0, std::min<long long>(knob(KNOB_VERIFY_MID_GENS), 64));
    r.tri_max = (uint32_t)std::max<long long>(0, std::min<long long>(knob(KNOB_LAT_TRI_MAX), 1u << 30));
    r.host_parts = (size_t)std::max<long long>(2, std::min<long long>(knob(KNOB_HOST_PARTS), 64));
    r.force_redo = knob(KNOB_FORCE_REDO) != 0 ? 1u : 0u;
    r.recheck = knob(KNOB_TEST_RECHECK) != 0 ? 1u : 0u;
    r.skip_flag = (uint32_t)std::max<long long>(0, std::min<long long>(knob(KNOB_TEST_SKIP_FLAG), 64));
    r.delay_x = (uint32_t)std::max<long long>(0, std::min<long long>(knob(KNOB_TEST_DELAY_X), 4096));
    return r;
  }
};
inline int overlap_parts(const Route& rt, size_t n) {
  if (rt.overlap >= 0) return (int)std::min<long long>(rt.overlap, 64);
  return n > CHUNK ? 2 : 0;
}

void resident_stop(Dev& d);  // single.hip

// ------------------------------------------------------------------ device registry (engine.hip)
extern std::mutex g_mu;
extern std::vector<DevPtr> g_devs;
extern bool g_inited;

inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

struct DevGuard {  // restores the caller's current device
  int prev = -1;
  explicit DevGuard(int d) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    (void)hipSetDevice(d);
  }
  ~DevGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

int ensure_buf(uint8_t*& buf, size_t& cap_io, hipStream_t st, hipEvent_t last, size_t bytes, size_t min_cap);
int dev_ensure_buf(Dev& d, size_t bytes);
int init_device(int id, DevPtr* out);
int ensure_init();
DevPtr dev_by_id(int id);
DevPtr first_dev();
size_t dev_ws_bytes(const Dev& d);

// Enqueue on `st` after all previous engine work on this device; record completion.
struct Serial {
  Dev& d;
  hipStream_t st;
  Serial(Dev& dev, hipStream_t s) : d(dev), st(s) { (void)hipStreamWaitEvent(st, d.last, 0); }
  ~Serial() { (void)hipEventRecord(d.last, st); }
};

// Device-wide work (lane-serial and mid-size batches, the device-resident entries, synthesis):
// counted in d.wide first, so the resident server can be neither handed a job nor relaunched
// from then on; then the server is stopped (it would otherwise hold CUs the device-wide kernels
// are sized for) and the device mutex taken.
struct DeviceWide {
  Dev& d;
  std::unique_lock<std::mutex> lk;
  explicit DeviceWide(Dev& dv) : d(dv) {
    d.wide.fetch_add(1, std::memory_order_acq_rel);
    resident_stop(d);
    lk = std::unique_lock<std::mutex>(d.mu);
  }
  ~DeviceWide() {
    lk.unlock();
    d.wide.fetch_sub(1, std::memory_order_acq_rel);
  }
};

// The device's diagnostic counters and the test-only knobs, on every launch's parameters.
template <class P>
P with_diag(const Dev& d, P p, const Route& rt) {
  p.diag = d.diag;
  p.force_redo = rt.force_redo;
  p.test_skip_flag = rt.skip_flag;
  p.test_skip_block = 0;
  if constexpr (std::is_same<P, RecoverParams>::value) p.test_delay_x = rt.delay_x;
  return p;
}

// One recover pass over prepared records: the latency kernel for small passes, else the
// resident-grid lane-serial kernel (its workspace bound checked by the launcher).
// ------------------------------------------------------------------ routing (route.hip)
bool mid_bucket(const Dev& d, const Route& rt, size_t n);
bool use_mid(const Dev& d, const Route& rt, size_t n);
bool mid_bkt2(const Dev& d, const Route& rt, size_t n);
bool verify_mid(const Dev& d, const Route& rt, size_t n);
hipError_t launch_verify_any(Dev& d, const Route& rt, const VerifyParams& p, bool small, hipStream_t st);
bool fused_parse(const Dev& d, const Route& rt, size_t n);
bool sender_fused(const Dev& d, const Route& rt, size_t n, std::initializer_list<const void*> rows);
void bind_sender_rows(RecoverParams& p, const uint8_t* h, const uint8_t* r, const uint8_t* s, const uint8_t* v,
                      const uint8_t* f, int signer, uint64_t chain_id);
// gens > 0: a lane-serial launch covers at most `gens` resident generations (host-buffer chunks,
// EGES_HOST_GENS) instead of the device's EGES_GRID_MULT
hipError_t launch_recover_pass(Dev& d, const Route& rt, const RecoverParams& p0, hipStream_t st, int gens = 0);
// wire-format rows after the recovery records (tx_rows_kernel's decode)
inline size_t tx_rows_bytes(size_t m) { return align_up(m * (4 * 32 + 1), 256); }
bool wire_fused(const Dev& d, const Route& rt, size_t m, const uint8_t* raw);
// the device's second compute stream and workspace (overlapped launches), created on first use
int ensure_aux(Dev& d);
// device-resident pipelines: all pointers device pointers, d.mu held by the caller
int run_recover_dev(Dev& d, const Route& rt, const uint8_t* msg, const uint8_t* sig, size_t n, uint8_t* pub,
                    uint8_t* addr, uint8_t* status, hipStream_t st);
int run_sender_dev(Dev& d, const Route& rt, const uint8_t* sighash, const uint8_t* r, const uint8_t* s, const uint8_t* v,
                   const uint8_t* vflags, size_t n, int signer, uint64_t chain_id, uint8_t* addr, uint8_t* status,
                   hipStream_t st);
int run_sender_raw_dev(Dev& d, const Route& rt, const uint8_t* raw, const uint64_t* offsets, size_t n, int signer, uint64_t chain_id,
                       uint8_t* addr, uint8_t* status, uint8_t* sighash_out, hipStream_t st);
int run_precompile_dev(Dev& d, const Route& rt, const uint8_t* input, const uint32_t* inlen, size_t n, uint8_t* out32, uint8_t* status,
                       hipStream_t st);
int run_verify_dev(Dev& d, const Route& rt, const uint8_t* pub, const uint8_t* publen, const uint8_t* msg, const uint8_t* sig, size_t n,
                   uint8_t* ok, hipStream_t st);

// ------------------------------------------------------------------ host-buffer paths (hostpath.hip)

// Copies the inputs of [off, off+cnt) to device scratch, runs, copies outputs back. Synchronous.
struct HostJob {
  enum Kind { RECOVER, SENDER, VERIFY, SENDER_RAW, PRECOMPILE } kind;
  const uint32_t* inlen = nullptr;  // PRECOMPILE: optional input lengths
  const uint64_t* offsets = nullptr;  // SENDER_RAW: n + 1 entries
  uint8_t* sighash = nullptr;         // SENDER_RAW: optional output
  bool decode_only = false;           // SENDER_RAW: decode only; status receives the vflags
  // inputs
  const uint8_t *a = nullptr, *b = nullptr, *c = nullptr, *d = nullptr, *e = nullptr;
  int signer = 0;
  uint64_t chain_id = 0;
  // outputs
  uint8_t *pub = nullptr, *addr = nullptr, *status = nullptr;
};

// contiguous index shards across the engine's devices, one host thread per device
int run_host(const HostJob& j, size_t n);
// decode-only pass over wire-format transactions (the GPU decoder, no recovery)
int decode_check_raw(const uint8_t* raw, const uint64_t* offsets, size_t n, int signer, uint64_t chain_id, bool* bad);
// a Geec block's (extblock) three transaction lists: each list's offsets into the block
bool split_extblock(const uint8_t* b, size_t len, std::vector<uint64_t> offs[3]);
void keccakf_host(uint64_t st[25]);

// ------------------------------------------------------------------ single-item seam (single.hip)
// eges_ecdsa_recover / eges_ecdsa_verify's bodies: coalesced into shared groups (the resident
// server or a lane); the result as the reference's (1 / 0), an engine failure's text in t_err
int single_recover(unsigned char* pub65, const unsigned char* sig65, const unsigned char* msg32);
int single_verify(const unsigned char* sig64, const unsigned char* msg32, const unsigned char* pub, size_t publen);

}  // namespace eges::host
