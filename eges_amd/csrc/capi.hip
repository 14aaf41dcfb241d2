// C-ABI of libeges.so (include/eges.h): device management, staging, multi-GPU sharding.
//
// Replaces the reference's cgo seam (crypto/secp256k1/secp256.go:45-134, ext.h:18-75). There is
// no CPU compute path here: every recovery / verification runs on gfx950 through the kernels in
// k_*.hip, and the entries fail with EGES_E_NODEVICE when no such device is usable.
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

namespace {

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

thread_local std::string t_err;

inline void cpu_relax() {
#if defined(__x86_64__)
  __builtin_ia32_pause();
#else
  std::this_thread::yield();
#endif
}

int set_err(int rc, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  t_err = buf;
  return rc;
}

int env_int(const char* name, int dflt) {
  const char* e = std::getenv(name);
  return e && *e ? std::atoi(e) : dflt;
}

#define HIPCHK(expr)                                                                                \
  do {                                                                                              \
    hipError_t e_ = (expr);                                                                         \
    if (e_ != hipSuccess) return set_err(EGES_E_HIP, "%s failed: %s", #expr, hipGetErrorString(e_)); \
  } while (0)

// A small-call lane: its own stream, device scratch and pinned staging, so that concurrent
// single-chunk host calls that run on the latency kernel (which needs no shared workspace) do
// not queue behind each other on the device mutex.
constexpr int NLANES = 4;
// A host-buffer call's input gate (handoff.cuh gate_wait / gate_done): word 0 the last sequence
// opened, word 1 set by a wave whose wait ran out, word 2 the last completed sequence. Coherent
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

// ------------------------------------------------------------------ knobs (knobs.h)
// Name (the environment variable read once at the first eges_init) and product default.
struct KnobDef {
  const char* name;
  long long dflt;
};
// Batches (or pipeline chunks) of at most LAT_MAX signatures run on the latency kernels
// (k_recover_lat.hip: one signature per wave), up to MID_MAX on the mid-size kernel
// (k_recover_mid.hip), larger ones on the lane-serial throughput kernel. Cuts from C1-shaped
// whole calls (tools/gpu_latcut.sh).
// Overlapped launches (OVERLAP): a device-resident recover batch runs as launches alternating
// between two streams with their own workspaces, so each launch's tail (its slowest waves)
// overlaps the next launch's start. Auto (-1): on when the batch spans more than one CHUNK (64M
// signatures: +3.9 % on one box), off for a single-chunk batch, whose launch then stays one
// kernel. S >= 2 forces S parts; 0 turns it off.
#ifndef EGES_LAT_MAX_DEFAULT
#define EGES_LAT_MAX_DEFAULT 1536
#endif
#ifndef EGES_MID_MAX_DEFAULT
#define EGES_MID_MAX_DEFAULT 40000
#endif
const KnobDef KNOB_DEFS[] = {
    {"EGES_LAT_MAX", EGES_LAT_MAX_DEFAULT},
    {"EGES_LAT_WIDE_MAX", 256},
    {"EGES_MID_MAX", EGES_MID_MAX_DEFAULT},
    {"EGES_MID_FORM", 1},
    {"EGES_WIRE_FUSED", 1},
    {"EGES_TXROWS_WAVE_MAX", 8192},
    {"EGES_TEST_ROOT_HELPERS", 1},
    {"EGES_OVERLAP", -1},
    {"EGES_TEST_FORCE_REDO", 0},
    {"EGES_COALESCE_GATHER_US", 20},
    {"EGES_COALESCE_SPIN_US", 2000},
    {"EGES_COALESCE_SPINNERS", 8},
    {"EGES_SENDER_FUSED", 1},
    {"EGES_LAT_TRI_MAX", 448},
    {"EGES_HOST_PARTS", EGES_PIPE_PARTS},
    {"EGES_TEST_SKIP_FLAG", 0},
    {"EGES_TEST_DELAY_X", 0},
    {"EGES_RESIDENT", 1},
    {"EGES_RESIDENT_WGS", 16},
    {"EGES_RESIDENT_CAP", 64},
    {"EGES_RESIDENT_IDLE_MS", 4},
    {"EGES_GATE", 1},
};
static_assert(sizeof(KNOB_DEFS) / sizeof(KNOB_DEFS[0]) == KNOB_COUNT, "a name and default for every knob");
std::atomic<long long> g_knob[KNOB_COUNT];
std::once_flag g_knob_once;

void knobs_load_env() {  // once per process, from eges_init (the only getenv of these names)
  std::call_once(g_knob_once, [] {
    for (int k = 0; k < KNOB_COUNT; ++k) {
      const char* e = std::getenv(KNOB_DEFS[k].name);
      g_knob[k].store(e && *e ? std::strtoll(e, nullptr, 10) : KNOB_DEFS[k].dflt, std::memory_order_relaxed);
    }
  });
}
int knob_index(const char* name) {
  if (!name) return -1;
  for (int k = 0; k < KNOB_COUNT; ++k)
    if (std::strcmp(name, KNOB_DEFS[k].name) == 0) return k;
  return -1;
}

// The routing knobs of one call, read once at its start (a knob flipped while a call
// runs must not send part of it one way and part another, e.g. a small-lane call onto the
// windowed form's shared workspace).
struct Route {
  size_t lat_max = 0, mid_max = 0;
  uint32_t wide_max = 0, tri_max = 0;
  long long mid_form = 1, wire_fused = 1, overlap = -1, sender_fused = 1, gate = 1;
  size_t host_parts = EGES_PIPE_PARTS;
  uint32_t force_redo = 0, skip_flag = 0, delay_x = 0;
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
    r.tri_max = (uint32_t)std::max<long long>(0, std::min<long long>(knob(KNOB_LAT_TRI_MAX), 1u << 30));
    r.host_parts = (size_t)std::max<long long>(2, std::min<long long>(knob(KNOB_HOST_PARTS), 64));
    r.force_redo = knob(KNOB_FORCE_REDO) != 0 ? 1u : 0u;
    r.skip_flag = (uint32_t)std::max<long long>(0, std::min<long long>(knob(KNOB_TEST_SKIP_FLAG), 64));
    r.delay_x = (uint32_t)std::max<long long>(0, std::min<long long>(knob(KNOB_TEST_DELAY_X), 4096));
    return r;
  }
};
static int overlap_parts(const Route& rt, size_t n) {
  if (rt.overlap >= 0) return (int)std::min<long long>(rt.overlap, 64);
  return n > CHUNK ? 2 : 0;
}

void resident_stop(Dev& d);

std::mutex g_mu;
std::vector<DevPtr> g_devs;
bool g_inited = false;

size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

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

int ensure_buf(uint8_t*& buf, size_t& cap_io, hipStream_t st, hipEvent_t last, size_t bytes, size_t min_cap) {
  if (bytes <= cap_io) return EGES_SUCCESS;
  if (buf) {
    HIPCHK(hipStreamSynchronize(st));
    if (last) HIPCHK(hipEventSynchronize(last));
    HIPCHK(hipFree(buf));
    buf = nullptr;
    cap_io = 0;
  }
  size_t cap = std::max(bytes, min_cap);
  if (hipMalloc(&buf, cap) != hipSuccess) return set_err(EGES_E_NOMEM, "hipMalloc(%zu) failed", cap);
  cap_io = cap;
  return EGES_SUCCESS;
}
int dev_ensure_buf(Dev& d, size_t bytes) { return ensure_buf(d.buf, d.buf_cap, d.stream, d.last, bytes, size_t(64) << 20); }

int init_device(int id, DevPtr* out) {
  hipDeviceProp_t prop;
  HIPCHK(hipGetDeviceProperties(&prop, id));
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return set_err(EGES_E_NODEVICE, "device %d is %s, the engine is built for gfx950 only", id, prop.gcnArchName);
  DevGuard g(id);
  DevPtr d = std::make_shared<Dev>();
  d->id = id;
  d->cus = prop.multiProcessorCount;
  // the small-call lanes' streams first: HIP hands out its hardware queues (GPU_MAX_HW_QUEUES,
  // 4 by default) round-robin in stream-creation order, and lanes sharing a queue serialise
  for (Lane& l : d->lanes) {
    HIPCHK(hipStreamCreateWithFlags(&l.stream, hipStreamNonBlocking));
    for (int r = 0; r < 2; ++r) {
      HIPCHK(hipEventCreateWithFlags(&l.ev_in[r], hipEventDisableTiming));
      HIPCHK(hipEventCreateWithFlags(&l.ev_k[r], hipEventDisableTiming));
    }
  }
  HIPCHK(hipStreamCreateWithFlags(&d->stream, hipStreamNonBlocking));
  HIPCHK(hipEventCreateWithFlags(&d->last, hipEventDisableTiming));
  HIPCHK(hipStreamCreateWithFlags(&d->copy, hipStreamNonBlocking));
  for (int r = 0; r < 2; ++r) {
    HIPCHK(hipEventCreateWithFlags(&d->ev_in[r], hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&d->ev_k[r], hipEventDisableTiming));
  }
  // Lane-serial grids of two resident generations (EGES_GRID_MULT, default 2): a 1M-signature
  // pass then gives 4 signatures per thread instead of 8, and the blocks of the second
  // generation start as the first generation's finish, filling the tail the slowest waves leave
  // (the batch inversions, amortised over 4 instead of 8, cost less than that tail): C2 +2.0 %
  // (99.4 -> 101.3 M sigs/s, 3 reps each, same box), C4 +0.1 %, VerifySignature +1.2 %.
  const int gm = std::max(1, std::min(8, env_int("EGES_GRID_MULT", 2)));
  d->mb_recover = occupancy_recover() * d->cus * gm;
  d->mb_verify = occupancy_verify() * d->cus * gm;
  d->mb_synth = occupancy_synth() * d->cus;
  if (const int cap = env_int("EGES_TEST_MAX_BLOCKS", 0); cap > 0) {  // tests: a small device
    d->mb_recover = std::min(d->mb_recover, cap);
    d->mb_verify = std::min(d->mb_verify, cap);
    d->mb_synth = std::min(d->mb_synth, cap);
  }
  // A full pass may need more blocks than are resident (grid_for_lane_serial caps the
  // signatures per thread at MAX_SLOTS): the workspace covers the larger of the two.
  const int mb = std::max(d->mb_recover, std::max(d->mb_verify, d->mb_synth));
  d->ws_blocks = std::max(mb, std::max(lane_serial_grid((uint32_t)CHUNK, d->mb_recover),
                                       lane_serial_grid((uint32_t)CHUNK, d->mb_verify)));
  HIPCHK(hipMalloc(&d->gtab, gtab_bytes()));
  HIPCHK(hipMalloc(&d->ws, ws_bytes_per_block() * (size_t)d->ws_blocks));
  HIPCHK(hipMalloc(&d->diag, DIAG_WORDS * sizeof(uint32_t)));
  HIPCHK(hipMemsetAsync(d->diag, 0, DIAG_WORDS * sizeof(uint32_t), d->stream));
  HIPCHK(launch_init_gtab(d->gtab, d->stream));
  HIPCHK(hipEventRecord(d->last, d->stream));
  HIPCHK(hipStreamSynchronize(d->stream));
  *out = std::move(d);
  return EGES_SUCCESS;
}

// Resources go when the last reference does: eges_shutdown drops the registry's references,
// and a call still in flight keeps its device alive until it returns.
Dev::~Dev() {
  DevGuard g(id);
  resident_stop(*this);  // (its stream is lane 0's)
  if (res.job) (void)hipHostFree(res.job);
  if (res.data) (void)hipHostFree(res.data);
  if (res.counter) (void)hipFree(res.counter);
  if (stream) (void)hipStreamSynchronize(stream);
  if (last) (void)hipEventSynchronize(last);  // the last engine work, on whichever stream the caller gave
  if (gtab) (void)hipFree(gtab);
  if (ws) (void)hipFree(ws);
  if (diag) (void)hipFree(diag);
  if (buf) (void)hipFree(buf);
  if (pin) (void)hipHostFree(pin);
  if (gate.w) (void)hipHostFree(gate.w);
  if (vfault) (void)hipHostFree(vfault);
  if (gate.dev) (void)hipFree(gate.dev);
  if (last) (void)hipEventDestroy(last);
  for (int r = 0; r < 2; ++r) {
    if (ev_in[r]) (void)hipEventDestroy(ev_in[r]);
    if (ev_k[r]) (void)hipEventDestroy(ev_k[r]);
  }
  if (copy) (void)hipStreamDestroy(copy);
  if (aux) {
    (void)hipStreamSynchronize(aux);
    (void)hipStreamDestroy(aux);
    (void)hipEventDestroy(ev_fork);
    (void)hipEventDestroy(ev_join);
    (void)hipFree(ws2);
  }
  for (Lane& l : lanes) {
    if (l.stream) (void)hipStreamSynchronize(l.stream);
    if (l.buf) (void)hipFree(l.buf);
    if (l.pin) (void)hipHostFree(l.pin);
    if (l.vfault) (void)hipHostFree(l.vfault);
    for (int r = 0; r < 2; ++r) {
      if (l.ev_in[r]) (void)hipEventDestroy(l.ev_in[r]);
      if (l.ev_k[r]) (void)hipEventDestroy(l.ev_k[r]);
    }
    if (l.stream) (void)hipStreamDestroy(l.stream);
  }
  if (stream) (void)hipStreamDestroy(stream);
}

int ensure_init() {
  {
    std::lock_guard<std::mutex> lk(g_mu);
    if (g_inited && !g_devs.empty()) return EGES_SUCCESS;
  }
  int rc = eges_init(0, 0);
  return rc;
}

DevPtr dev_by_id(int id) {
  std::lock_guard<std::mutex> lk(g_mu);
  for (const DevPtr& d : g_devs)
    if (d->id == id) return d;
  return nullptr;
}

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
#ifdef EGES_PHASE_STAMPS
static uint64_t* g_stamps = nullptr;
static size_t g_stamp_waves = 0, g_stamp_cap = 0;
static hipError_t stamp_buf(size_t waves, hipStream_t st) {
  if (waves > g_stamp_cap) {
    if (g_stamps) (void)hipFree(g_stamps);
    g_stamps = nullptr;
    g_stamp_cap = 0;
    hipError_t e = hipMalloc(&g_stamps, waves * 8 * sizeof(uint64_t));
    if (e != hipSuccess) return e;
    g_stamp_cap = waves;
  }
  g_stamp_waves = waves;
  return hipMemsetAsync(g_stamps, 0, waves * 8 * sizeof(uint64_t), st);
}
#endif

size_t dev_ws_bytes(const Dev& d) { return ws_bytes_per_block() * (size_t)d.ws_blocks; }

// Host-side phase stamps of the last host-buffer call (diagnostic build only, tools/block_bench):
// 0 entry, 1 lane / device acquired, 2 inputs packed, 3 launches enqueued, 4 streams drained,
// 5 outputs unpacked (steady_clock, ns).
#ifdef EGES_PHASE_STAMPS
static int64_t g_hstamp[6];
#define HSTAMP(k) (g_hstamp[k] = std::chrono::steady_clock::now().time_since_epoch().count())
extern "C" size_t eges_diag_host_stamps(int64_t* out, size_t n) {
  for (size_t k = 0; k < n && k < 6; ++k) out[k] = g_hstamp[k];
  return 6;
}
#else
#define HSTAMP(k) ((void)0)
#endif
// batches (or chunks) the mid-size kernel takes: above LAT_MAX, up to MID_MAX and what the
// device workspace holds
// The bucket form (k_recover_mid.hip) holds 138 KB of LDS: one workgroup per CU. It is the
// faster form while the grid fits one generation (n <= 64 x CUs); beyond that the windowed form
// (two workgroups per CU) is (tools/formcurve.py).
bool mid_bucket(const Dev& d, const Route& rt, size_t n) {
  const long long f = rt.mid_form;
  if (f == 0) return false;
  if (f >= 2) return true;
  return (n + MID_SIGS_PER_BLOCK - 1) / MID_SIGS_PER_BLOCK <= (size_t)d.cus;
}
bool use_mid(const Dev& d, const Route& rt, size_t n) {
  if (n <= rt.lat_max || n > rt.mid_max) return false;
  return mid_bucket(d, rt, n) || (n + 63) / 64 * mid_ws_bytes_per_block() <= dev_ws_bytes(d);
}
// VerifySignature batches above LAT_MAX that the bucket form's verify mode takes (one generation of
// workgroups: n <= 64 x CUs), instead of the lane-serial verify kernel's fixed chain
bool verify_mid(const Dev& d, const Route& rt, size_t n) {
  return rt.mid_form != 0 && n > rt.lat_max && n <= rt.mid_max &&
         (n + MID_SIGS_PER_BLOCK - 1) / MID_SIGS_PER_BLOCK <= (size_t)d.cus;
}
hipError_t launch_verify_any(Dev& d, const Route& rt, const VerifyParams& p, bool small, hipStream_t st) {
  if (small || p.n <= rt.lat_max) return launch_verify_lat(p, p.n <= rt.wide_max, st);
  if (verify_mid(d, rt, p.n)) return launch_verify_mid(p, st);
  return launch_verify(p, d.mb_verify, d.ws_blocks, st);
}
// the recover kernels that parse msg / sig bytes themselves (no prep launch)
bool fused_parse(const Dev& d, const Route& rt, size_t n) { return n <= rt.lat_max || use_mid(d, rt, n); }
// ... and classify types.Sender rows themselves (no prep_sender launch): 4-byte aligned rows only
bool sender_fused(const Dev& d, const Route& rt, size_t n, std::initializer_list<const void*> rows) {
  if (rt.sender_fused == 0 || !fused_parse(d, rt, n)) return false;
  for (const void* q : rows)
    if (((uintptr_t)q & 3u) != 0) return false;
  return true;
}
void bind_sender_rows(RecoverParams& p, const uint8_t* h, const uint8_t* r, const uint8_t* s, const uint8_t* v,
                      const uint8_t* f, int signer, uint64_t chain_id) {
  p.snd_h = h;
  p.snd_r = r;
  p.snd_s = s;
  p.snd_v = v;
  p.snd_f = f;
  p.snd_signer = signer;
  p.snd_chain_id = chain_id;
}

hipError_t launch_recover_pass(Dev& d, const Route& rt, const RecoverParams& p0, hipStream_t st) {
  RecoverParams p = with_diag(d, p0, rt);
  // the split form (four waves per signature) while the batch leaves SIMDs idle, then the
  // three-wave form, then the narrow form (k_recover_lat.hip FORM_*)
  // (the three-wave form only while its workgroups and the root helpers, three waves each, fit
  // one generation at its occupancy of 3 waves per SIMD)
  const bool tri = p.n <= rt.tri_max && 3 * (size_t)p.n + 3 * ((p.n + 127) / 128) <= (size_t)d.cus * 4 * 3;
  p.wide = p.n <= rt.wide_max ? 1u : tri ? 2u : 0u;
  const bool mid = use_mid(d, rt, p.n);
  if (p.wire_raw && !(mid ? mid_bucket(d, rt, p.n) : p.n <= rt.lat_max)) return hipErrorInvalidValue;  // wire_fused() decides
  if (p.snd_r && !(mid || p.n <= rt.lat_max)) return hipErrorInvalidValue;  // sender_fused() decides
  if (p.gate && !mid) return hipErrorInvalidValue;  // (the host waits for the mid-size kernels' completion word)
#ifdef EGES_PHASE_STAMPS
  if (mid) {
    hipError_t e = stamp_buf((p.n + 63) / 64 * 4, st);  // one row per wave
    return e != hipSuccess ? e : launch_recover_mid_stamped(p, mid_bucket(d, rt, p.n), dev_ws_bytes(d), st, g_stamps);
  }
  if (p.n <= rt.lat_max || p.raw_sig) {
    hipError_t e = stamp_buf(lat_waves(p.n), st);
    return e != hipSuccess ? e : launch_recover_lat_stamped(p, st, g_stamps);
  }
#endif
  if (mid) return launch_recover_mid(p, mid_bucket(d, rt, p.n), dev_ws_bytes(d), st);
  if (p.n <= rt.lat_max || p.raw_sig) return launch_recover_lat(p, st);
  return launch_recover(p, d.mb_recover, d.ws_blocks, st);
}

// ------------------------------------------------------------------ device-side pipelines
// All pointers device pointers; d.mu held by the caller.
#ifdef EGES_PHASE_STAMPS
// Diagnostic build (libeges_diag.so): per-wave phase cycle sums of the last recover launch.
extern "C" size_t eges_diag_read_stamps(uint64_t* out, size_t max_waves) {
  const size_t w = g_stamp_waves < max_waves ? g_stamp_waves : max_waves;
  if (g_stamps && out && w) {
    if (hipDeviceSynchronize() != hipSuccess) return 0;
    if (hipMemcpy(out, g_stamps, w * 8 * sizeof(uint64_t), hipMemcpyDeviceToHost) != hipSuccess) return 0;
  }
  return w;
}
#endif

// the device's second compute stream and workspace (overlapped launches), created on first use
int ensure_aux(Dev& d) {
  if (d.aux) return EGES_SUCCESS;
  HIPCHK(hipStreamCreateWithFlags(&d.aux, hipStreamNonBlocking));
  HIPCHK(hipEventCreateWithFlags(&d.ev_fork, hipEventDisableTiming));
  HIPCHK(hipEventCreateWithFlags(&d.ev_join, hipEventDisableTiming));
  HIPCHK(hipMalloc(&d.ws2, ws_bytes_per_block() * (size_t)d.ws_blocks));
  return EGES_SUCCESS;
}

int run_recover_dev_overlap(Dev& d, const Route& rt, const uint8_t* msg, const uint8_t* sig, size_t n, uint8_t* pub, uint8_t* addr,
                            uint8_t* status, hipStream_t st, int parts) {
  const size_t per = std::min(CHUNK, (n + parts - 1) / parts);
  const size_t n_pad = align_up(per, 64);
  const size_t region = align_up(recover_scratch_bytes(n_pad), 256);
  int rc = dev_ensure_buf(d, 2 * region);
  if (rc) return rc;
  if ((rc = ensure_aux(d))) return rc;
  Serial ser(d, st);
  HIPCHK(hipEventRecord(d.ev_fork, st));
  HIPCHK(hipStreamWaitEvent(d.aux, d.ev_fork, 0));
  int j = 0;
  for (size_t off = 0; off < n; off += per, ++j) {
    const uint32_t m = (uint32_t)std::min(per, n - off);
    hipStream_t sj = (j & 1) ? d.aux : st;
    uint32_t* rec = reinterpret_cast<uint32_t*>(d.buf + (j & 1) * region);
    HIPCHK(launch_prep_ecrecover(msg + off * 32, sig + off * 65, m, (uint32_t)n_pad, rec, sj));
    RecoverParams p{rec, m, (uint32_t)n_pad, status + off, addr ? addr + off * 20 : nullptr, pub ? pub + off * 65 : nullptr,
                    d.gtab, (j & 1) ? d.ws2 : d.ws};
    HIPCHK(launch_recover(with_diag(d, p, rt), d.mb_recover, d.ws_blocks, sj));
  }
  HIPCHK(hipEventRecord(d.ev_join, d.aux));
  HIPCHK(hipStreamWaitEvent(st, d.ev_join, 0));
  return EGES_SUCCESS;
}

int run_recover_dev(Dev& d, const Route& rt, const uint8_t* msg, const uint8_t* sig, size_t n, uint8_t* pub,
                    uint8_t* addr, uint8_t* status, hipStream_t st) {
  const int parts = overlap_parts(rt, n);
  if (parts >= 2 && n >= (size_t)parts * 64 * 1024)
    return run_recover_dev_overlap(d, rt, msg, sig, n, pub, addr, status, st, parts);
  const size_t c = std::min(n, CHUNK);
  const size_t n_pad = align_up(c, 64);
  int rc = dev_ensure_buf(d, recover_scratch_bytes(n_pad));
  if (rc) return rc;
  uint32_t* rec = reinterpret_cast<uint32_t*>(d.buf);
  Serial ser(d, st);
  for (size_t off = 0; off < n; off += CHUNK) {
    const uint32_t m = (uint32_t)std::min(CHUNK, n - off);
    RecoverParams p{rec, m, (uint32_t)n_pad, status + off, addr ? addr + off * 20 : nullptr, pub ? pub + off * 65 : nullptr,
                    d.gtab, d.ws};
    if (fused_parse(d, rt, m)) {  // the latency / mid-size kernels parse the bytes themselves
      p.raw_msg = msg + off * 32;
      p.raw_sig = sig + off * 65;
    } else {
      HIPCHK(launch_prep_ecrecover(msg + off * 32, sig + off * 65, m, (uint32_t)n_pad, rec, st));
    }
#ifdef EGES_PHASE_STAMPS
    if (!fused_parse(d, rt, p.n)) {
      HIPCHK(stamp_buf((size_t)d.ws_blocks * 4 /* waves per block */, st));
      HIPCHK(launch_recover_stamped(with_diag(d, p, rt), d.mb_recover, d.ws_blocks, st, g_stamps));
      continue;
    }
#endif
    HIPCHK(launch_recover_pass(d, rt, p, st));
  }
  return EGES_SUCCESS;
}

int run_sender_dev(Dev& d, const Route& rt, const uint8_t* sighash, const uint8_t* r, const uint8_t* s, const uint8_t* v,
                   const uint8_t* vflags, size_t n, int signer, uint64_t chain_id, uint8_t* addr, uint8_t* status,
                   hipStream_t st) {
  const size_t c = std::min(n, CHUNK);
  const size_t n_pad = align_up(c, 64);
  int rc = dev_ensure_buf(d, recover_scratch_bytes(n_pad));
  if (rc) return rc;
  uint32_t* rec = reinterpret_cast<uint32_t*>(d.buf);
  Serial ser(d, st);
  for (size_t off = 0; off < n; off += CHUNK) {
    const uint32_t m = (uint32_t)std::min(CHUNK, n - off);
    RecoverParams p{rec, m, (uint32_t)n_pad, status + off, addr + off * 20, nullptr, d.gtab, d.ws};
    const uint8_t *h_ = sighash + off * 32, *r_ = r + off * 32, *s_ = s + off * 32, *v_ = v + off * 32;
    const uint8_t* f_ = vflags ? vflags + off : nullptr;
    if (sender_fused(d, rt, m, {h_, r_, s_, v_}))
      bind_sender_rows(p, h_, r_, s_, v_, f_, signer, chain_id);
    else
      HIPCHK(launch_prep_sender(h_, r_, s_, v_, f_, m, (uint32_t)n_pad, signer, chain_id, rec, st));
    HIPCHK(launch_recover_pass(d, rt, p, st));
  }
  return EGES_SUCCESS;
}

// Wire-format transactions: tx_rows_kernel (decode + sighash) writes the sender rows into device
// scratch after the recovery records; then the sender pipeline runs unchanged.
inline size_t tx_rows_bytes(size_t m) { return align_up(m * (4 * 32 + 1), 256); }
// Batches the bucket form or the latency kernels take run their wire-format decode, sighash and
// Sender checks inside the recovery kernel (RecoverParams::wire_*): no tx_rows / prep_sender
// launches and no rows in between. EGES_WIRE_FUSED: 1 both (default), 2 the bucket form only,
// 0 neither (A/B and tests).
bool wire_fused(const Dev& d, const Route& rt, size_t m, const uint8_t* raw) {
  const long long f = rt.wire_fused;
  if (f == 0 || ((uintptr_t)raw & 3u) != 0) return false;
  return (f == 1 && m <= rt.lat_max) || (use_mid(d, rt, m) && mid_bucket(d, rt, m));
}

int run_sender_raw_dev(Dev& d, const Route& rt, const uint8_t* raw, const uint64_t* offsets, size_t n, int signer, uint64_t chain_id,
                       uint8_t* addr, uint8_t* status, uint8_t* sighash_out, hipStream_t st) {
  const size_t c = std::min(n, CHUNK);
  const size_t n_pad = align_up(c, 64);
  const size_t o_rows = align_up(recover_scratch_bytes(n_pad), 256);
  int rc = dev_ensure_buf(d, o_rows + tx_rows_bytes(c));
  if (rc) return rc;
  uint32_t* rec = reinterpret_cast<uint32_t*>(d.buf);
  uint8_t* rows = d.buf + o_rows;
  Serial ser(d, st);
  for (size_t off = 0; off < n; off += CHUNK) {
    const uint32_t m = (uint32_t)std::min(CHUNK, n - off);
    uint8_t* hs = sighash_out ? sighash_out + off * 32 : rows;
    uint8_t* rr = rows + (size_t)m * 32;
    uint8_t* sr = rr + (size_t)m * 32;
    uint8_t* vr = sr + (size_t)m * 32;
    uint8_t* vf = vr + (size_t)m * 32;
    RecoverParams p{rec, m, (uint32_t)n_pad, status + off, addr + off * 20, nullptr, d.gtab, d.ws};
    if (wire_fused(d, rt, m, raw)) {
      p.wire_raw = raw;
      p.wire_off = offsets;
      p.wire_first = off;
      p.wire_signer = signer;
      p.wire_chain_id = chain_id;
      p.wire_sighash = sighash_out ? hs : nullptr;
    } else {
      HIPCHK(launch_tx_rows(raw, offsets, off, m, signer, chain_id, hs, rr, sr, vr, vf, st));
      HIPCHK(launch_prep_sender(hs, rr, sr, vr, vf, m, (uint32_t)n_pad, signer, chain_id, rec, st));
    }
    HIPCHK(launch_recover_pass(d, rt, p, st));
  }
  return EGES_SUCCESS;
}

// EVM precompile: 32-byte output words (12 zero bytes + address) written in place by the
// recover kernel (addr_stride 32) after the words are cleared.
int run_precompile_dev(Dev& d, const Route& rt, const uint8_t* input, const uint32_t* inlen, size_t n, uint8_t* out32, uint8_t* status,
                       hipStream_t st) {
  const size_t c = std::min(n, CHUNK);
  const size_t n_pad = align_up(c, 64);
  int rc = dev_ensure_buf(d, recover_scratch_bytes(n_pad));
  if (rc) return rc;
  uint32_t* rec = reinterpret_cast<uint32_t*>(d.buf);
  Serial ser(d, st);
  HIPCHK(hipMemsetAsync(out32, 0, n * 32, st));
  for (size_t off = 0; off < n; off += CHUNK) {
    const uint32_t m = (uint32_t)std::min(CHUNK, n - off);
    HIPCHK(launch_prep_precompile(input + off * 128, inlen ? inlen + off : nullptr, m, (uint32_t)n_pad, rec, st));
    RecoverParams p{rec, m, (uint32_t)n_pad, status + off, out32 + off * 32 + 12, nullptr, d.gtab, d.ws, 32};
    HIPCHK(launch_recover_pass(d, rt, p, st));
  }
  return EGES_SUCCESS;
}

int run_verify_dev(Dev& d, const Route& rt, const uint8_t* pub, const uint8_t* publen, const uint8_t* msg, const uint8_t* sig, size_t n,
                   uint8_t* ok, hipStream_t st) {
  const size_t n_pad = align_up(std::min(n, CHUNK), 64);
  int rc = dev_ensure_buf(d, verify_scratch_bytes(n_pad));
  if (rc) return rc;
  Serial ser(d, st);
  for (size_t off = 0; off < n; off += CHUNK) {
    const uint32_t m = (uint32_t)std::min(CHUNK, n - off);
    VerifyParams p{pub + off * 65, publen + off, msg + off * 32, sig + off * 64, m, ok + off, d.gtab, d.ws};
    verify_scratch_bind(p, d.buf, n_pad);
    p = with_diag(d, p, rt);
    HIPCHK(launch_verify_any(d, rt, p, false, st));
  }
  return EGES_SUCCESS;
}

// ------------------------------------------------------------------ host-buffer pipelines
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

// Device bytes of one pipeline region for a chunk of m items: inputs | scratch | outputs.
struct Region {
  size_t in_bytes = 0, raw_lo = 0, raw_len = 0, o_rec = 0, o_out = 0, total = 0;
};
Region region_for(const HostJob& j, size_t base, size_t m) {
  Region g;
  const size_t m_pad = align_up(m, 64);
  switch (j.kind) {
    case HostJob::RECOVER: g.in_bytes = m * (32 + 65); break;
    case HostJob::SENDER: g.in_bytes = m * (32 * 4 + 1); break;
    case HostJob::VERIFY: g.in_bytes = m * (65 + 1 + 32 + 64); break;
    case HostJob::PRECOMPILE: g.in_bytes = m * (128 + 4); break;
    case HostJob::SENDER_RAW:
      g.raw_lo = j.offsets[base] - j.offsets[0];
      g.raw_len = j.offsets[base + m] - j.offsets[base];
      g.in_bytes = align_up(g.raw_len, 8) + 8 * (m + 1) + tx_rows_bytes(m);
      break;
  }
  const size_t rec_bytes = (j.kind == HostJob::VERIFY) ? verify_scratch_bytes(m_pad) : recover_scratch_bytes(m_pad);
  g.o_rec = align_up(g.in_bytes, 256);
  g.o_out = g.o_rec + align_up(rec_bytes, 256);
  g.total = align_up(g.o_out + m * (65 + 32 + 1), 256);
  return g;
}

// Host-buffer pipeline over chunks of one shard. Two device regions alternate: while the
// compute stream runs chunk i, the copy stream stages chunk i+1's inputs and returns chunk
// i-1's outputs (host order H2D(i+1), K(i+1), D2H(i): the pageable D2H blocks this thread
// until K(i) is done, by which time K(i+1) is queued behind it). Synchronous overall.
int run_host_shard(Dev& d, const Route& rt, const HostJob& j, size_t off, size_t cnt) {
  HSTAMP(0);
  DevGuard g(d.id);
  // a shard big enough to pipeline runs as >= 2 chunks (each still a full resident grid)
  size_t c = std::min(CHUNK, cnt);
  if (cnt >= 2 * PIPE_MIN && c > cnt / 2)
    c = std::min(CHUNK, std::max(PIPE_MIN / 2, align_up((cnt + rt.host_parts - 1) / rt.host_parts, 64)));
  size_t worst = 0;  // region size: SENDER_RAW depends on the bytes of each chunk
  for (size_t base = off; base < off + cnt; base += c) worst = std::max(worst, region_for(j, base, std::min(c, off + cnt - base)).total);
  const int nreg = cnt > c ? 2 : 1;
  const bool pinned = nreg == 1 && worst <= PIN_BYTES;
  // Small calls on the latency kernel (no shared workspace) run on one of the device's lanes,
  // concurrently with each other; everything else on the device's main resources, in order.
  const bool small = pinned && cnt <= rt.lat_max;
  Lane* lane = nullptr;
  std::unique_lock<std::mutex> lk;
  std::unique_ptr<DeviceWide> wide;
  if (small) {
    for (Lane& l : d.lanes) {
      std::unique_lock<std::mutex> t(l.mu, std::try_to_lock);
      if (t.owns_lock() && !l.reserved.load(std::memory_order_acquire)) {
        lane = &l;
        lk = std::move(t);
        break;
      }
    }
    while (!lane) {
      static std::atomic<unsigned> rr{0};
      Lane& l = d.lanes[rr++ % NLANES];
      std::unique_lock<std::mutex> t(l.mu);
      if (l.reserved.load(std::memory_order_acquire)) continue;  // (the resident server's)
      lane = &l;
      lk = std::move(t);
    }
  } else {
    wide = std::make_unique<DeviceWide>(d);  // device-wide work: the resident server leaves the CUs first
  }
  uint8_t*& dbuf = small ? lane->buf : d.buf;
  uint8_t*& pin = small ? lane->pin : d.pin;
  hipEvent_t* ev_in = small ? lane->ev_in : d.ev_in;
  hipEvent_t* ev_k = small ? lane->ev_k : d.ev_k;
  int rc = small ? ensure_buf(lane->buf, lane->buf_cap, lane->stream, nullptr, worst, size_t(4) << 20)
                 : dev_ensure_buf(d, worst * nreg);
  if (rc) return rc;
  // a single chunk has nothing to overlap: one stream, no cross-stream waits (C3 latency)
  hipStream_t st = small ? lane->stream : d.stream, sx = nreg > 1 ? d.copy : st;
  // Every return after this point (errors included) first drains every stream, so the lane /
  // device mutex is never released while kernels or copies of this call still touch its
  // pinned staging or scratch (the next caller writes its inputs there).
  struct Drain {
    hipStream_t a, b;
    bool armed;
    ~Drain() {
      if (!armed) return;
      (void)hipStreamSynchronize(a);
      if (b != a) (void)hipStreamSynchronize(b);
    }
  } drain{st, sx, true};
  if (pinned && !pin && hipHostMalloc(&pin, PIN_BYTES, hipHostMallocDefault) != hipSuccess) {
    pin = nullptr;
    return set_err(EGES_E_NOMEM, "hipHostMalloc(%zu) failed", PIN_BYTES);
  }
  // A pinned call whose mid-size kernel reads the inputs itself (the fused bucket / windowed forms)
  // launches first and copies its inputs into the pinned buffer while the launch is in flight:
  // the kernels wait at the gate (handoff.cuh gate_wait), which opens after the copies. Opening is
  // also the guard's destructor, so no return path leaves a launched kernel waiting (declared
  // after `drain`: it runs first).
  Gate& gate = d.gate;  // (the mid-size kernels run above EGES_LAT_MAX: never on a lane)
  const bool gating = pinned && !small && rt.gate != 0 &&
                      (j.kind == HostJob::RECOVER || j.kind == HostJob::SENDER || (j.kind == HostJob::SENDER_RAW && !j.decode_only));
  if (gating && !gate.w) {
    if (hipHostMalloc(&gate.w, 64, hipHostMallocCoherent) != hipSuccess) {
      gate.w = nullptr;
      return set_err(EGES_E_NOMEM, "hipHostMalloc(gate) failed");
    }
    std::memset(gate.w, 0, 64);
    if (hipMalloc(&gate.dev, 64) != hipSuccess || hipMemset(gate.dev, 0, 64) != hipSuccess) {
      (void)hipHostFree(gate.w);
      gate.w = nullptr;
      gate.dev = nullptr;
      return set_err(EGES_E_NOMEM, "hipMalloc(gate) failed");
    }
  }
  struct GateOpen {
    struct Copy {
      uint8_t* dst;
      const void* src;
      size_t n;
    } q[8];
    int nq = 0;
    uint32_t* w = nullptr;  // armed: the kernels wait for sequence `seq`
    uint32_t seq = 0;
    void open() {
      for (int i = 0; i < nq; ++i) std::memcpy(q[i].dst, q[i].src, q[i].n);
      nq = 0;
      if (w) __atomic_store_n(w, seq, __ATOMIC_RELEASE);
      w = nullptr;
    }
    ~GateOpen() { open(); }
  } gopen;
  bool defer = false;  // this chunk's inputs wait for gopen.open()
  bool gated = false;  // a gated mid-size launch ran: its last workgroup stores the sequence into gate.w[2]
  auto arm = [&](RecoverParams& p) {  // a deferred chunk's kernels wait at the gate
    if (!defer || p.n == 0) return;
    if (++gate.seq == 0) gate.seq = 1;
    gated = true;  // (a mid-size launch: its kernels store the completion word)
    p.gate = gate.w;
    p.gate_dev = gate.dev;
    p.gate_seq = gate.seq;
    gopen.w = gate.w;
    gopen.seq = gate.seq;
  };
  // VerifySignature: a hand-off fault leaves its item's ok byte 0 and stores 1 into this word
  uint32_t*& vfault = small ? lane->vfault : d.vfault;
  if (j.kind == HostJob::VERIFY) {
    if (!vfault && hipHostMalloc(&vfault, 64, hipHostMallocCoherent) != hipSuccess) {
      vfault = nullptr;
      return set_err(EGES_E_NOMEM, "hipHostMalloc(fault word) failed");
    }
    __atomic_store_n(vfault, 0u, __ATOMIC_RELAXED);
  }
  if (!small) {
    HIPCHK(hipStreamWaitEvent(st, d.last, 0));
    HIPCHK(hipStreamWaitEvent(sx, d.last, 0));
  }
  HSTAMP(1);
  // Input staging: each input array goes to its offset in the region, either by its own
  // (pageable) copy into device memory on the copy stream, or, for a pinned call, packed into
  // the pinned buffer at the same offset, where the kernels read it directly (zero-copy: no
  // H2D / D2H operations at all, the outputs are written straight into the pinned buffer too).
  auto h2d = [&](uint8_t* B, uint8_t* dst, const void* src, size_t bytes) -> int {
    if (!bytes) return EGES_SUCCESS;
    if (pinned) {  // dst points into the pinned buffer (see I below)
      if (defer && gopen.nq < 8) gopen.q[gopen.nq++] = {dst, src, bytes};
      else std::memcpy(dst, src, bytes);  // (at most 5 inputs per kind: q never fills)
      return EGES_SUCCESS;
    }
    (void)B;
    HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, sx));
    return EGES_SUCCESS;
  };
  auto flush_in = [&](uint8_t*) -> int { return EGES_SUCCESS; };
#define H2D(B, dst, src, bytes)                   \
  do {                                             \
    int rc_ = h2d((B), (dst), (src), (bytes));     \
    if (rc_) return rc_;                           \
  } while (0)
#define FLUSH_IN(B)                 \
  do {                              \
    int rc_ = flush_in(B);          \
    if (rc_) return rc_;            \
    HSTAMP(2);                      \
  } while (0)
  // the kernels wait for their inputs' copies (a single chunk uses one stream: nothing to join)
#define JOIN_IN(r)                                      \
  do {                                                  \
    if (sx != st) {                                     \
      HIPCHK(hipEventRecord(ev_in[r], sx));             \
      HIPCHK(hipStreamWaitEvent(sk, ev_in[r], 0));      \
    }                                                   \
  } while (0)
  struct Pending {
    size_t base, m;
    int r;
    uint8_t* B;
    Region g;
  };
  const size_t astride = j.kind == HostJob::PRECOMPILE ? 32 : 20;
  auto sighash_off = [&](const Pending& q) { return align_up(q.g.raw_len, 8) + 8 * (q.m + 1); };
  auto outputs = [&](const Pending& q) -> int {  // D2H of one chunk, on the copy stream
    uint8_t* o_pub = q.B + q.g.o_out;
    uint8_t* o_addr = o_pub + q.m * 65;
    uint8_t* o_st = o_addr + q.m * 32;
    if (sx != st) HIPCHK(hipStreamWaitEvent(sx, ev_k[q.r], 0));
    if (pinned) {  // outputs are already in the pinned buffer; the signing hashes are not
      if (j.kind == HostJob::SENDER_RAW && j.sighash)
        HIPCHK(hipMemcpyAsync(pin + sighash_off(q), q.B + sighash_off(q), q.m * 32, hipMemcpyDeviceToHost, sx));
      return EGES_SUCCESS;
    }
    if (j.pub) HIPCHK(hipMemcpyAsync(j.pub + q.base * 65, o_pub, q.m * 65, hipMemcpyDeviceToHost, sx));
    if (j.addr) HIPCHK(hipMemcpyAsync(j.addr + q.base * astride, o_addr, q.m * astride, hipMemcpyDeviceToHost, sx));
    if (j.status) HIPCHK(hipMemcpyAsync(j.status + q.base, o_st, q.m, hipMemcpyDeviceToHost, sx));
    if (j.kind == HostJob::SENDER_RAW && j.sighash)
      HIPCHK(hipMemcpyAsync(j.sighash + q.base * 32, q.B + sighash_off(q), q.m * 32, hipMemcpyDeviceToHost, sx));
    return EGES_SUCCESS;
  };
  auto unpack = [&](const Pending& q) {  // pinned mode, after the sync
    const uint8_t* o_pub = pin + q.g.o_out;
    const uint8_t* o_addr = o_pub + q.m * 65;
    const uint8_t* o_st = o_addr + q.m * 32;
    if (j.pub) std::memcpy(j.pub + q.base * 65, o_pub, q.m * 65);
    if (j.addr) std::memcpy(j.addr + q.base * astride, o_addr, q.m * astride);
    if (j.status) std::memcpy(j.status + q.base, o_st, q.m);
    if (j.kind == HostJob::SENDER_RAW && j.sighash) std::memcpy(j.sighash + q.base * 32, pin + sighash_off(q), q.m * 32);
  };
  Pending prev{};
  bool have_prev = false;
  int ci = 0;
  for (size_t base = off; base < off + cnt; base += c, ++ci) {
    const size_t m = std::min(c, off + cnt - base);
    const size_t m_pad = align_up(m, 64);
    const int r = ci % nreg;
    hipStream_t sk = st;  // this chunk's compute stream
    uint32_t* wsk = d.ws;
    const Region rg = region_for(j, base, m);
    uint8_t* B = dbuf + (size_t)r * worst;
    uint8_t* I = pinned ? pin : B;  // where the kernels read the inputs
    uint8_t* o_pub = (pinned ? pin : B) + rg.o_out;
    uint8_t* o_addr = o_pub + m * 65;
    uint8_t* o_st = o_addr + m * 32;
    uint32_t* rec = reinterpret_cast<uint32_t*>(B + rg.o_rec);
    // --- inputs (copy stream), then the kernels (compute stream)
    if (j.kind == HostJob::RECOVER) {
      uint8_t* dm = I;
      uint8_t* ds = dm + m * 32;
      const bool fused = fused_parse(d, rt, m);
      defer = gating && fused && use_mid(d, rt, m);  // (the latency kernels measured +-0 to +1.5 % slower)
      H2D(B, dm, j.a + base * 32, m * 32);
      H2D(B, ds, j.b + base * 65, m * 65);
      FLUSH_IN(B);
      JOIN_IN(r);
      RecoverParams p{rec, (uint32_t)m, (uint32_t)m_pad, o_st, j.addr ? o_addr : nullptr, j.pub ? o_pub : nullptr,
                      d.gtab, wsk};
      if (fused) {  // the latency / mid-size kernels parse the bytes themselves
        p.raw_msg = dm;
        p.raw_sig = ds;
      } else {
        HIPCHK(launch_prep_ecrecover(dm, ds, (uint32_t)m, (uint32_t)m_pad, rec, sk));
      }
      arm(p);
      HIPCHK(launch_recover_pass(d, rt, p, sk));
    } else if (j.kind == HostJob::SENDER) {
      uint8_t* dh = I;
      uint8_t* dr = dh + m * 32;
      uint8_t* dsv = dr + m * 32;
      uint8_t* dv = dsv + m * 32;
      uint8_t* df = dv + m * 32;
      const bool fused = sender_fused(d, rt, m, {dh, dr, dsv, dv});
      defer = gating && fused && use_mid(d, rt, m);  // (the latency kernels measured +-0 to +1.5 % slower)
      H2D(B, dh, j.a + base * 32, m * 32);
      H2D(B, dr, j.b + base * 32, m * 32);
      H2D(B, dsv, j.c + base * 32, m * 32);
      H2D(B, dv, j.d + base * 32, m * 32);
      if (j.e) H2D(B, df, j.e + base, m);
      FLUSH_IN(B);
      JOIN_IN(r);
      RecoverParams p{rec, (uint32_t)m, (uint32_t)m_pad, o_st, o_addr, nullptr, d.gtab, wsk};
      if (fused)  // the recover kernel reads the rows itself
        bind_sender_rows(p, dh, dr, dsv, dv, j.e ? df : nullptr, j.signer, j.chain_id);
      else
        HIPCHK(launch_prep_sender(dh, dr, dsv, dv, j.e ? df : nullptr, (uint32_t)m, (uint32_t)m_pad, j.signer, j.chain_id,
                                  rec, sk));
      arm(p);
      HIPCHK(launch_recover_pass(d, rt, p, sk));
    } else if (j.kind == HostJob::PRECOMPILE) {
      uint8_t* din = I;
      uint32_t* dlen = reinterpret_cast<uint32_t*>(din + m * 128);
      H2D(B, din, j.a + base * 128, m * 128);
      if (j.inlen) H2D(B, reinterpret_cast<uint8_t*>(dlen), j.inlen + base, m * 4);
      FLUSH_IN(B);
      JOIN_IN(r);
      if (pinned) std::memset(o_addr, 0, m * 32);
      else HIPCHK(hipMemsetAsync(o_addr, 0, m * 32, sk));
      HIPCHK(launch_prep_precompile(din, j.inlen ? dlen : nullptr, (uint32_t)m, (uint32_t)m_pad, rec, sk));
      RecoverParams p{rec, (uint32_t)m, (uint32_t)m_pad, o_st, o_addr + 12, nullptr, d.gtab, wsk, 32};
      HIPCHK(launch_recover_pass(d, rt, p, sk));
    } else if (j.kind == HostJob::SENDER_RAW) {
      uint8_t* draw = I;
      uint64_t* doff = reinterpret_cast<uint64_t*>(draw + align_up(rg.raw_len, 8));
      uint8_t* hs = B + align_up(rg.raw_len, 8) + 8 * (m + 1);  // decoded rows: device memory
      uint8_t* rr = hs + m * 32;
      uint8_t* sr = rr + m * 32;
      uint8_t* vr = sr + m * 32;
      uint8_t* vf = vr + m * 32;
      // (the fused form reads the encodings straight from the pinned buffer: a pipelined host copy
      // + DMA into device memory measured 0.486-0.508 ms against 0.450 ms for C1, same kernel)
      const bool fused = !j.decode_only && wire_fused(d, rt, m, draw);
      defer = gating && fused && use_mid(d, rt, m);  // (the latency kernels measured +-0 to +1.5 % slower)
      if (rg.raw_len) H2D(B, draw, j.a + rg.raw_lo, rg.raw_len);
      H2D(B, reinterpret_cast<uint8_t*>(doff), j.offsets + base, 8 * (m + 1));
      FLUSH_IN(B);
      JOIN_IN(r);
      if (j.decode_only) {  // the decoder's flags straight into the status bytes
        HIPCHK(launch_tx_rows(draw, doff, 0, (uint32_t)m, j.signer, j.chain_id, hs, rr, sr, vr, o_st, sk));
      } else {
        RecoverParams p{rec, (uint32_t)m, (uint32_t)m_pad, o_st, o_addr, nullptr, d.gtab, wsk};
        if (fused) {
          p.wire_raw = draw;
          p.wire_off = doff;
          p.wire_signer = j.signer;
          p.wire_chain_id = j.chain_id;
          p.wire_sighash = j.sighash ? hs : nullptr;
        } else {
          HIPCHK(launch_tx_rows(draw, doff, 0, (uint32_t)m, j.signer, j.chain_id, hs, rr, sr, vr, vf, sk));
          HIPCHK(launch_prep_sender(hs, rr, sr, vr, vf, (uint32_t)m, (uint32_t)m_pad, j.signer, j.chain_id, rec, sk));
        }
        arm(p);
        HIPCHK(launch_recover_pass(d, rt, p, sk));
      }
    } else {
      uint8_t* dp = I;
      uint8_t* dl = dp + m * 65;
      uint8_t* dm = dl + m;
      uint8_t* ds = dm + m * 32;
      H2D(B, dp, j.a + base * 65, m * 65);
      H2D(B, dl, j.b + base, m);
      H2D(B, dm, j.c + base * 32, m * 32);
      H2D(B, ds, j.d + base * 64, m * 64);
      FLUSH_IN(B);
      JOIN_IN(r);
      VerifyParams p{dp, dl, dm, ds, (uint32_t)m, o_st, d.gtab, wsk};
      verify_scratch_bind(p, B + rg.o_rec, m_pad);
      p = with_diag(d, p, rt);
      p.fault = vfault;
      // small (lane) calls must not touch the device's shared workspace: latency kernel
      HIPCHK(launch_verify_any(d, rt, p, small, sk));
    }
    HSTAMP(3);
    if (defer) gopen.open();  // the inputs, while the launch is in flight; then the gate
    defer = false;
    if (sx != st) HIPCHK(hipEventRecord(ev_k[r], sk));
    // --- the previous chunk's outputs, while this chunk computes
    if (have_prev) {
      rc = outputs(prev);
      if (rc) return rc;
    }
    prev = Pending{base, m, r, B, rg};
    have_prev = true;
  }
  if (have_prev) {
    rc = outputs(prev);
    if (rc) return rc;
  }
  if (!small) HIPCHK(hipEventRecord(d.last, sx));
  // a gated single launch with nothing queued behind it: its completion word instead of the
  // stream's completion signal (handoff.cuh gate_done); later work on the stream stays ordered
  // after it, and nothing of this call reads the pinned buffer any more once the word is set
  bool done = false;
  if (gated && nreg == 1 && !(j.kind == HostJob::SENDER_RAW && j.sighash)) {
    const auto t0 = std::chrono::steady_clock::now();
    for (uint64_t spins = 0; !(done = __atomic_load_n(&gate.w[2], __ATOMIC_ACQUIRE) == gate.seq); ++spins) {
      cpu_relax();
      if ((spins & 1023) == 1023 && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) break;
    }
    if (done) (void)hipStreamQuery(st);  // (lets the runtime retire the launch)
  }
  if (!done) {
    HIPCHK(hipStreamSynchronize(sx));
    if (sx != st) HIPCHK(hipStreamSynchronize(st));  // (st's last work is already behind sx's events)
    if (gated && __atomic_load_n(&gate.w[2], __ATOMIC_ACQUIRE) != gate.seq) {
      (void)hipMemset(gate.dev + 1, 0, 4);  // (the workgroup count, for the next call)
      return set_err(EGES_E_HIP, "a gated launch ended without its completion word");
    }
  }
  HSTAMP(4);
  drain.armed = false;
  if (gating && __atomic_load_n(&gate.w[1], __ATOMIC_ACQUIRE) != 0u) {
    __atomic_store_n(&gate.w[1], 0u, __ATOMIC_RELAXED);
    return set_err(EGES_E_HIP, "a kernel's input gate timed out");
  }
  if (pinned && have_prev) unpack(prev);
  HSTAMP(5);
  if (j.kind == HostJob::VERIFY && __atomic_load_n(vfault, __ATOMIC_ACQUIRE) != 0u)
    return set_err(EGES_E_HIP, "a kernel hand-off timed out (items read invalid; EGES_DIAG_HANDOFF)");
  // items a kernel marked EGES_ENGINE_FAULT (a wave hand-off timed out, handoff.cuh) have no
  // result: the call fails rather than return them
  if (j.status && !j.decode_only && std::memchr(j.status + off, EGES_ENGINE_FAULT, cnt))
    return set_err(EGES_E_HIP, "a kernel hand-off timed out (EGES_ENGINE_FAULT items; EGES_DIAG_HANDOFF)");
  return EGES_SUCCESS;
#undef H2D
#undef FLUSH_IN
#undef JOIN_IN
}

// Contiguous index shards across the engine's devices.
int run_host(const HostJob& j, size_t n) {
  if (n == 0) return EGES_SUCCESS;
  int rc = ensure_init();
  if (rc) return rc;
  std::vector<DevPtr> devs;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    devs = g_devs;
  }
  if (devs.empty()) return set_err(EGES_E_NODEVICE, "no gfx950 device available");
  const Route rt = Route::now();
  // small batches stay on one device (a Geec block of 1000 txs is one tile set)
  size_t ndev = std::min(devs.size(), std::max<size_t>(1, n / 65536));
  const size_t per = (n + ndev - 1) / ndev;
  if (ndev == 1) return run_host_shard(*devs[0], rt, j, 0, n);
  std::vector<int> rcs(ndev, EGES_SUCCESS);
  std::vector<std::string> errs(ndev);
  std::vector<std::thread> th;
  for (size_t i = 0; i < ndev; ++i) {
    const size_t lo = i * per, hi = std::min(n, lo + per);
    if (lo >= hi) continue;
    th.emplace_back([&, i, lo, hi] {
      rcs[i] = run_host_shard(*devs[i], rt, j, lo, hi - lo);
      if (rcs[i]) errs[i] = t_err;
    });
  }
  for (auto& t : th) t.join();
  for (size_t i = 0; i < ndev; ++i)
    if (rcs[i]) return set_err(rcs[i], "device %d: %s", devs[i]->id, errs[i].c_str());
  return EGES_SUCCESS;
}

// Decode-only pass over wire-format transactions (the same GPU decoder as eges_sender_raw_batch,
// no recovery): *bad = some item fails rlp.DecodeBytes.
int decode_check_raw(const uint8_t* raw, const uint64_t* offsets, size_t n, int signer, uint64_t chain_id, bool* bad) {
  *bad = false;
  if (n == 0) return EGES_SUCCESS;
  std::vector<uint8_t> vf(n);
  HostJob j;
  j.kind = HostJob::SENDER_RAW;
  j.decode_only = true;
  j.a = raw;
  j.offsets = offsets;
  j.signer = signer;
  j.chain_id = chain_id;
  j.status = vf.data();
  const int rc = run_host(j, n);
  if (rc) return rc;
  for (uint8_t f : vf)
    if (f & VF_DECODE_ERR) *bad = true;
  return EGES_SUCCESS;
}

// ------------------------------------------------------------------ Geec block (extblock) split
// RLP item header at b[p] inside [p, end) (rlp/decode.go readKind :937-990 and the Kind bound
// checks :874-907): kind 0 = byte, 1 = string, 2 = list; hl = header length, sz = payload size.
bool rlp_head(const uint8_t* b, size_t p, size_t end, int& kind, size_t& hl, size_t& sz) {
  if (p >= end) return false;  // EOL / EOF
  const uint8_t x = b[p];
  if (x < 0x80) {
    kind = 0;
    hl = 1;
    sz = 0;
    return true;
  }
  size_t ll = 0;
  if (x < 0xB8) {
    kind = 1;
    sz = x - 0x80u;
  } else if (x < 0xC0) {
    kind = 1;
    ll = x - 0xB7u;
  } else if (x < 0xF8) {
    kind = 2;
    sz = x - 0xC0u;
  } else {
    kind = 2;
    ll = x - 0xF7u;
  }
  hl = 1 + ll;
  if (ll) {  // readUint: big-endian length, no leading zero byte, and >= 56 (ErrCanonSize)
    if (p + 1 + ll > end || b[p + 1] == 0) return false;
    sz = 0;
    for (size_t k = 0; k < ll; ++k) sz = (sz << 8) | b[p + 1 + k];
    if (sz < 56) return false;
  }
  return sz <= end - p - hl;  // ErrElemTooLarge / ErrValueTooLarge
}

// The extblock list (core/types/block.go:188-195: Header, FakeTxs, GeecTxs, Txs, Uncles,
// Confirm rlp:"nil") of a whole block as rlp.DecodeBytes sees its structure: exactly six
// elements, the first five lists, the last empty or a list, no trailing bytes. Fills, for
// the three transaction lists, the item offsets (absolute in b; n_k + 1 each). Header, uncle
// and confirm-message field contents are not decoded (not on the signature path).
bool split_extblock(const uint8_t* b, size_t len, std::vector<uint64_t> offs[3]) {
  int kind;
  size_t hl, sz;
  if (!rlp_head(b, 0, len, kind, hl, sz) || kind != 2 || hl + sz != len) return false;
  size_t p = hl;
  const size_t end = len;
  for (int e = 0; e < 6; ++e) {
    if (!rlp_head(b, p, end, kind, hl, sz)) return false;
    if (e < 5 && kind != 2) return false;                      // Header, tx lists, Uncles: lists
    if (e == 5 && !(kind == 2 || (kind == 1 && sz == 0))) return false;  // *ConfirmBlockMsg, rlp:"nil"
    if (e >= 1 && e <= 3) {                                     // FakeTxs, GeecTxs, Txs
      std::vector<uint64_t>& o = offs[e - 1];
      o.clear();
      size_t q = p + hl;
      const size_t le = p + hl + sz;
      o.push_back(q);
      while (q < le) {
        int k2;
        size_t h2, s2;
        if (!rlp_head(b, q, le, k2, h2, s2)) return false;
        q += h2 + s2;
        o.push_back(q);
      }
    }
    p += hl + sz;
  }
  return p == end;  // "input list has too many elements"
}

// ------------------------------------------------------------------ host Keccak-256
const uint64_t RC[24] = {0x0000000000000001ULL, 0x0000000000008082ULL, 0x800000000000808AULL, 0x8000000080008000ULL,
                         0x000000000000808BULL, 0x0000000080000001ULL, 0x8000000080008081ULL, 0x8000000000008009ULL,
                         0x000000000000008AULL, 0x0000000000000088ULL, 0x0000000080008009ULL, 0x000000008000000AULL,
                         0x000000008000808BULL, 0x800000000000008BULL, 0x8000000000008089ULL, 0x8000000000008003ULL,
                         0x8000000000008002ULL, 0x8000000000000080ULL, 0x000000000000800AULL, 0x800000008000000AULL,
                         0x8000000080008081ULL, 0x8000000000008080ULL, 0x0000000080000001ULL, 0x8000000080008008ULL};
// rho offsets in the pi-permuted visiting order of the lane walk x,y -> y,2x+3y
const int ROTC[24] = {1, 3, 6, 10, 15, 21, 28, 36, 45, 55, 2, 14, 27, 41, 56, 8, 25, 43, 62, 18, 39, 61, 20, 44};
const int PILN[24] = {10, 7, 11, 17, 18, 3, 5, 16, 8, 21, 24, 4, 15, 23, 19, 13, 12, 2, 20, 14, 22, 9, 6, 1};

inline uint64_t rol(uint64_t x, int s) { return (x << s) | (x >> (64 - s)); }

void keccakf_host(uint64_t st[25]) {
  for (int round = 0; round < 24; ++round) {
    uint64_t bc[5];
    for (int i = 0; i < 5; ++i) bc[i] = st[i] ^ st[i + 5] ^ st[i + 10] ^ st[i + 15] ^ st[i + 20];
    for (int i = 0; i < 5; ++i) {
      const uint64_t t = bc[(i + 4) % 5] ^ rol(bc[(i + 1) % 5], 1);
      for (int j = 0; j < 25; j += 5) st[j + i] ^= t;
    }
    uint64_t t = st[1];
    for (int i = 0; i < 24; ++i) {
      const int j = PILN[i];
      const uint64_t tmp = st[j];
      st[j] = rol(t, ROTC[i]);
      t = tmp;
    }
    for (int j = 0; j < 25; j += 5) {
      for (int i = 0; i < 5; ++i) bc[i] = st[j + i];
      for (int i = 0; i < 5; ++i) st[j + i] ^= (~bc[(i + 1) % 5]) & bc[(i + 2) % 5];
    }
    st[0] ^= RC[round];
  }
}

// ------------------------------------------------------------------ single-item coalescing
// The reference's single-item calls (secp256k1_ext_ecdsa_recover / _verify, ext.h:30-75) run on
// one shared read-only context from any goroutine (secp256.go:45-52). Here concurrent single-item
// callers are coalesced ("group commit"): a caller enqueues its request; if no batch is in
// flight it becomes the leader, takes every queued request (its own included) and runs them as
// one batch (the latency kernel for small batches); the others wait on a condition variable and
// are served by that batch or the next one. Nothing is serialised per request.
struct RecoverReq {
  const uint8_t* msg;
  const uint8_t* sig;
  uint8_t* pub;
  int result = 0;
  int rc = EGES_SUCCESS;  // the group's engine call; nonzero: result 0 is an engine failure
  std::string err;        //   and its error text, for the caller's eges_last_error
  std::atomic<bool> done{false};
  std::atomic<bool> queued{false};
};
struct VerifyReq {
  const uint8_t* sig;
  const uint8_t* msg;
  const uint8_t* pub;
  uint8_t publen;
  int result = 0;
  int rc = EGES_SUCCESS;
  std::string err;
  std::atomic<bool> done{false};
  std::atomic<bool> queued{false};
};

// ------------------------------------------------------------------ resident single-call server
// Stops the device's resident server (before device-wide work, which it would otherwise share the
// CUs with, and at teardown): the stop word, then its stream drains.
void resident_halt(Dev& d, Resident& r) {  // r.mu held
  if (!r.running) return;
  DevGuard g(d.id);
  __atomic_store_n(&r.job->stop, 1u, __ATOMIC_RELEASE);
  (void)hipStreamSynchronize(r.stream);
  __atomic_store_n(&r.job->stop, 0u, __ATOMIC_RELEASE);
  r.running = false;
  d.lanes[r.lane].reserved.store(false, std::memory_order_release);
}
void resident_stop(Dev& d) {
  std::lock_guard<std::mutex> lk(d.res.mu);
  resident_halt(d, d.res);
}

// One job on the resident server of device d: fill(data, job) writes the inputs, read(data)
// takes the outputs. Returns -1 when the server is off, busy or the group too large (the caller
// takes a lane), else an EGES status.
uint32_t resident_cap() { return (uint32_t)std::max<long long>(1, std::min<long long>(knob(KNOB_RESIDENT_CAP), 4096)); }
template <class Fill, class Read>
int resident_job(Dev& d, Resident& r, int kind, size_t n, Fill&& fill, Read&& read) {
  if (knob(KNOB_RESIDENT) == 0 || n == 0) return -1;
  // the test-only knobs act on launches: their runs take the lanes
  if (knob(KNOB_FORCE_REDO) != 0 || knob(KNOB_TEST_SKIP_FLAG) != 0 || knob(KNOB_ROOT_HELPERS) == 0) return -1;
  const uint32_t cap = resident_cap();
  if (n > cap) return -1;
  std::unique_lock<std::mutex> lk(r.mu, std::try_to_lock);
  if (!lk.owns_lock()) return -1;
  // device-wide work running or still queued: the lanes (checked under r.mu, which resident_stop
  // takes after raising d.wide, so no server starts once a device-wide call has begun)
  if (d.wide.load(std::memory_order_acquire) != 0 || hipEventQuery(d.last) != hipSuccess) return -1;
  DevGuard g(d.id);
  if (!r.job || r.cap < cap) {
    if (r.running) return -1;  // (a knob raised while it runs: the lanes until it exits)
    r.stream = d.lanes[r.lane].stream;
    if (!r.job) {
      if (hipHostMalloc(&r.job, 4096, hipHostMallocCoherent) != hipSuccess) return set_err(EGES_E_NOMEM, "hipHostMalloc(job)");
      std::memset(r.job, 0, 4096);
      HIPCHK(hipMalloc(&r.counter, RESIDENT_COUNTER_BYTES));
      HIPCHK(hipMemset(r.counter, 0, RESIDENT_COUNTER_BYTES));
    }
    if (r.data) (void)hipHostFree(r.data);
    r.data = nullptr;
    // the data area is ordinary (cacheable) pinned memory, like the lanes' staging: uncached
    // (coherent) memory made scattered reads one PCIe read per lane. The server orders it by
    // system-scope fences around each job (k_recover_lat.hip resident_next / resident_done);
    // only the job word is coherent.
    if (hipHostMalloc(&r.data, resident_layout(cap).total, hipHostMallocDefault) != hipSuccess)
      return set_err(EGES_E_NOMEM, "hipHostMalloc(resident data)");
    r.cap = cap;
  }
  const long long idle_ms = std::max<long long>(1, knob(KNOB_RESIDENT_IDLE_MS));
  const auto now = std::chrono::steady_clock::now();
  // a server idle for half its bound may be deciding to exit: restart it rather than race it
  if (r.running &&
      (hipStreamQuery(r.stream) == hipSuccess || now - r.last_use > std::chrono::microseconds(idle_ms * 500)))
    resident_halt(d, r);
  auto launch = [&]() -> int {
    if (!r.running) {  // the lane finishes what it runs and takes no more calls
      std::lock_guard<std::mutex> l0(d.lanes[r.lane].mu);
      d.lanes[r.lane].reserved.store(true, std::memory_order_release);
    }
    HIPCHK(hipMemsetAsync(r.counter, 0, RESIDENT_COUNTER_BYTES, r.stream));
    if (++r.inst == 0) r.inst = 1;
    ResidentParams rp{r.job, r.data, r.cap, __atomic_load_n(&r.job->done, __ATOMIC_ACQUIRE), r.counter,
                      (uint64_t)idle_ms * 100000ull, r.inst, d.gtab, d.diag};
    r.wgs = (uint32_t)std::max<long long>(1, std::min<long long>(knob(KNOB_RESIDENT_WGS), 1024));
    if (!r.data || !r.counter) return set_err(EGES_E_HIP, "resident server: buffers missing");
    if (launch_lat_resident(rp, r.wgs, r.stream) != hipSuccess) {
      r.running = false;
      d.lanes[r.lane].reserved.store(false, std::memory_order_release);
      return set_err(EGES_E_HIP, "resident server launch failed");
    }
    r.running = true;
    return EGES_SUCCESS;
  };
  if (!r.running) {
    const int rc = launch();
    if (rc) return rc;
  }
  fill(r.data, r.job);
  __atomic_store_n(&r.job->n, (uint32_t)n, __ATOMIC_RELAXED);
  __atomic_store_n(&r.job->kind, (uint32_t)kind, __ATOMIC_RELAXED);
  const uint32_t seq = ++r.seq;
  __atomic_store_n(&r.job->seq, seq, __ATOMIC_RELEASE);
  const auto t0 = std::chrono::steady_clock::now();
  for (uint64_t spins = 0; __atomic_load_n(&r.job->done, __ATOMIC_ACQUIRE) != seq; ++spins) {
    cpu_relax();
    if ((spins & 1023) != 1023) continue;
    if (hipStreamQuery(r.stream) == hipSuccess && __atomic_load_n(&r.job->done, __ATOMIC_ACQUIRE) != seq) {
      // the server exited without taking the job (its idle bound): a fresh one takes it (lane 0
      // stays reserved in between)
      const int rc = launch();
      if (rc) return rc;
    }
    if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) {
      resident_halt(d, r);
      return set_err(EGES_E_HIP, "resident server: job %u not served within 2 s", seq);
    }
  }
  read(r.data);
  r.last_use = std::chrono::steady_clock::now();
  return EGES_SUCCESS;
}
DevPtr first_dev() {
  std::lock_guard<std::mutex> lk(g_mu);
  return g_devs.empty() ? nullptr : g_devs[0];
}

void run_group(std::vector<RecoverReq*>& g) {
  const size_t n = g.size();
  if (ensure_init() == EGES_SUCCESS) {
    if (DevPtr d = first_dev()) {
      const ResidentLayout L = resident_layout(resident_cap());
      const int rc = resident_job(
          *d, d->res, RESIDENT_RECOVER, n,
          [&](uint8_t* D, ResidentJob*) {
            for (size_t i = 0; i < n; ++i) {
              std::memcpy(D + L.msg + i * 32, g[i]->msg, 32);
              std::memcpy(D + L.sig + i * 65, g[i]->sig, 65);
            }
          },
          [&](const uint8_t* D) {
            bool fault = false;
            for (size_t i = 0; i < n; ++i) fault = fault || D[L.status + i] == EGES_ENGINE_FAULT;
            const int rc2 = fault ? set_err(EGES_E_HIP, "a kernel hand-off timed out (EGES_ENGINE_FAULT items)") : EGES_SUCCESS;
            for (size_t i = 0; i < n; ++i) {
              const bool ok = rc2 == EGES_SUCCESS && D[L.status + i] == EGES_OK;
              if (ok) std::memcpy(g[i]->pub, D + L.pub + i * 65, 65);
              g[i]->result = ok ? 1 : 0;
              g[i]->rc = rc2;
              if (rc2) g[i]->err = t_err;
            }
          });
      if (rc >= 0) {
        if (rc)
          for (RecoverReq* q : g) q->result = 0, q->rc = rc, q->err = t_err;
        return;
      }
    }
  }
  std::vector<uint8_t> msg(n * 32), sig(n * 65), pub(n * 65), st(n);
  for (size_t i = 0; i < n; ++i) {
    std::memcpy(&msg[i * 32], g[i]->msg, 32);
    std::memcpy(&sig[i * 65], g[i]->sig, 65);
  }
  const int rc = eges_ecrecover_batch(msg.data(), sig.data(), n, pub.data(), nullptr, st.data());
  for (size_t i = 0; i < n; ++i) {
    const bool ok = rc == EGES_SUCCESS && st[i] == EGES_OK;
    if (ok) std::memcpy(g[i]->pub, &pub[i * 65], 65);
    g[i]->result = ok ? 1 : 0;
    g[i]->rc = rc;
    if (rc) g[i]->err = t_err;
  }
}
void run_group(std::vector<VerifyReq*>& g) {
  const size_t n = g.size();
  if (ensure_init() == EGES_SUCCESS) {
    if (DevPtr d = first_dev()) {
      const ResidentLayout L = resident_layout(resident_cap());
      const int rc = resident_job(
          *d, d->res, RESIDENT_VERIFY, n,
          [&](uint8_t* D, ResidentJob*) {
            *reinterpret_cast<uint32_t*>(D + L.vfault) = 0u;
            for (size_t i = 0; i < n; ++i) {
              std::memset(D + L.vpub + i * 65, 0, 65);
              std::memcpy(D + L.vpub + i * 65, g[i]->pub, g[i]->publen);
              D[L.vpublen + i] = g[i]->publen;
              std::memcpy(D + L.vmsg + i * 32, g[i]->msg, 32);
              std::memcpy(D + L.vsig + i * 64, g[i]->sig, 64);
            }
          },
          [&](const uint8_t* D) {
            const bool fault = *reinterpret_cast<const volatile uint32_t*>(D + L.vfault) != 0u;
            const int rc2 = fault ? set_err(EGES_E_HIP, "a kernel hand-off timed out (EGES_DIAG_HANDOFF)") : EGES_SUCCESS;
            for (size_t i = 0; i < n; ++i) {
              g[i]->result = (rc2 == EGES_SUCCESS && D[L.vok + i] == 1) ? 1 : 0;
              g[i]->rc = rc2;
              if (rc2) g[i]->err = t_err;
            }
          });
      if (rc >= 0) {
        if (rc)
          for (VerifyReq* q : g) q->result = 0, q->rc = rc, q->err = t_err;
        return;
      }
    }
  }
  std::vector<uint8_t> pub(n * 65, 0), publen(n), msg(n * 32), sig(n * 64), ok(n);
  for (size_t i = 0; i < n; ++i) {
    std::memcpy(&pub[i * 65], g[i]->pub, g[i]->publen);
    publen[i] = g[i]->publen;
    std::memcpy(&msg[i * 32], g[i]->msg, 32);
    std::memcpy(&sig[i * 64], g[i]->sig, 64);
  }
  const int rc = eges_verify_batch(pub.data(), publen.data(), msg.data(), sig.data(), n, ok.data());
  for (size_t i = 0; i < n; ++i) {
    g[i]->result = (rc == EGES_SUCCESS && ok[i]) ? 1 : 0;
    g[i]->rc = rc;
    if (rc) g[i]->err = t_err;
  }
}

// Up to NLANES groups are in flight at once (one per small-call lane of the device), so a
// caller that arrives while a group runs does not wait for it to finish before its own starts.
// Waiting callers spin on their own completion flag (a futex wake-up costs tens of µs against a
// ~0.15 ms call) and fall back to blocking after EGES_COALESCE_SPIN_US. One leader at a time
// gathers: for up to EGES_COALESCE_GATHER_US it waits until as many requests are queued as the
// previous group had (the callers of a group that just finished come back within microseconds,
// and one launch for all of them beats a launch for the first and a lane wait for the rest),
// while the callers it will take spin instead of leading groups of their own.
template <class Req>
struct Coalescer {
  static constexpr size_t MAX_GROUP = 4096;
  std::mutex mu;
  std::condition_variable cv;
  std::vector<Req*> queue;       // guarded by mu
  std::atomic<size_t> qlen{0};   // queue.size(), for the gathering leader
  std::atomic<int> inflight{0};  // groups running or gathering (changed under mu)
  std::atomic<bool> gathering{false};  // a leader is gathering (changed under mu)
  std::atomic<int> spinners{0};        // callers spinning on their completion flag
  size_t last_group = 1;         // guarded by mu

  static std::chrono::microseconds us_knob(KnobId k) {
    return std::chrono::microseconds(std::max<long long>(0, knob(k)));
  }
  bool may_lead(const Req* r) const {
    return r->queued.load(std::memory_order_relaxed) && inflight.load(std::memory_order_relaxed) < NLANES &&
           !gathering.load(std::memory_order_relaxed);
  }

  // mu held on entry and exit; the caller has counted this group in `inflight` and set `gathering`
  void lead(std::unique_lock<std::mutex>& lk) {
    const auto gather = us_knob(KNOB_COALESCE_GATHER_US);
    const size_t want = std::min(last_group, MAX_GROUP);
    if (queue.size() < want && gather.count() > 0) {
      lk.unlock();
      const auto deadline = std::chrono::steady_clock::now() + gather;
      while (qlen.load(std::memory_order_acquire) < want && std::chrono::steady_clock::now() < deadline) cpu_relax();
      lk.lock();
    }
    std::vector<Req*> g;
    const size_t take = std::min(queue.size(), MAX_GROUP);  // >= 1: the leader's own request is queued
    g.assign(queue.begin(), queue.begin() + take);
    queue.erase(queue.begin(), queue.begin() + take);
    qlen.store(queue.size(), std::memory_order_release);
    for (Req* q : g) q->queued.store(false, std::memory_order_relaxed);
    last_group = std::max<size_t>(1, take);
    gathering.store(false, std::memory_order_relaxed);
    if (!queue.empty()) cv.notify_all();  // a blocked caller may lead the next group
    lk.unlock();
    run_group(g);
    // a spinning caller returns as soon as its flag is set: the store is the last touch of q
    for (Req* q : g) q->done.store(true, std::memory_order_release);
    lk.lock();
    --inflight;
    cv.notify_all();
  }

  void submit(Req* r) {
    const auto spin = us_knob(KNOB_COALESCE_SPIN_US);
    const auto t0 = std::chrono::steady_clock::now();
    std::unique_lock<std::mutex> lk(mu);
    r->queued.store(true, std::memory_order_relaxed);
    queue.push_back(r);
    qlen.store(queue.size(), std::memory_order_release);
    for (;;) {
      if (r->done.load(std::memory_order_acquire)) return;
      if (may_lead(r)) {
        ++inflight;
        gathering.store(true, std::memory_order_relaxed);
        lead(lk);
        continue;
      }
      // served by another leader's group, or waiting for a free lane: spin, then block. At most
      // EGES_COALESCE_SPINNERS callers spin at once: with more spinning threads than the
      // process's CPUs the leaders that launch and collect the groups get descheduled
      const int max_spinners = (int)std::max<long long>(0, knob(KNOB_COALESCE_SPINNERS));
      lk.unlock();
      bool block = spinners.fetch_add(1, std::memory_order_relaxed) >= max_spinners;
      while (!block && !r->done.load(std::memory_order_acquire)) {
        if (may_lead(r)) break;
        if (std::chrono::steady_clock::now() - t0 > spin) {
          block = true;
          break;
        }
        cpu_relax();
      }
      spinners.fetch_sub(1, std::memory_order_relaxed);
      lk.lock();
      if (block) cv.wait(lk, [&] { return r->done.load() || may_lead(r); });
    }
  }
};
Coalescer<RecoverReq> g_recover_co;
Coalescer<VerifyReq> g_verify_co;

}  // namespace

namespace eges {
long long knob(KnobId k) { return g_knob[k].load(std::memory_order_relaxed); }
}  // namespace eges

// ====================================================================== C ABI
extern "C" {

int eges_abi_version(void) { return EGES_ABI_VERSION; }

const char* eges_last_error(void) { return t_err.c_str(); }

int eges_init(uint32_t device_mask, uint32_t flags) {
  (void)flags;
  knobs_load_env();
  std::lock_guard<std::mutex> lk(g_mu);
  if (g_inited && !g_devs.empty()) return EGES_SUCCESS;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count <= 0)
    return set_err(EGES_E_NODEVICE, "no HIP device visible");
  std::string errs;
  // tests only: register every device k times (independent streams / workspaces), so the
  // multi-device shard path of run_host runs on a one-GPU box
  const int logical = std::max(1, std::min(8, env_int("EGES_TEST_LOGICAL_DEVICES", 1)));
  for (int i = 0; i < count && i < 32; ++i) {
    if (device_mask && !((device_mask >> i) & 1u)) continue;
    for (int k = 0; k < logical; ++k) {
      DevPtr d;
      int rc = init_device(i, &d);
      if (rc == EGES_SUCCESS) g_devs.push_back(std::move(d));
      else errs += t_err + "; ";
    }
  }
  if (g_devs.empty()) return set_err(EGES_E_NODEVICE, "no usable gfx950 device (%s)", errs.c_str());
  g_inited = true;
  return EGES_SUCCESS;
}

void eges_shutdown(void) {
  std::vector<DevPtr> devs;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    devs.swap(g_devs);
    g_inited = false;
  }
  // each device is released once its in-flight calls (which hold references) have returned
  for (DevPtr& d : devs) {
    resident_stop(*d);
    { std::lock_guard<std::mutex> dl(d->mu); }
    d.reset();
  }
}

int eges_device_count(void) {
  std::lock_guard<std::mutex> lk(g_mu);
  return (int)g_devs.size();
}

int eges_ecrecover_batch(const uint8_t* msg, const uint8_t* sig, size_t n, uint8_t* pub_out, uint8_t* addr_out,
                         uint8_t* status) {
  if (n == 0) return EGES_SUCCESS;
  if (!msg || !sig) return set_err(EGES_E_NULLPTR, "msg/sig is NULL");
  std::vector<uint8_t> tmp;
  HostJob j;
  j.kind = HostJob::RECOVER;
  j.a = msg;
  j.b = sig;
  j.pub = pub_out;
  j.addr = addr_out;
  if (!status) {
    tmp.resize(n);
    status = tmp.data();
  }
  j.status = status;
  return run_host(j, n);
}

int eges_sender_batch(const uint8_t* sighash, const uint8_t* r, const uint8_t* s, const uint8_t* v, const uint8_t* vflags,
                      size_t n, int signer, uint64_t chain_id, uint8_t* addr_out, uint8_t* status) {
  if (n == 0) return EGES_SUCCESS;
  if (!sighash || !r || !s || !v || !addr_out || !status) return set_err(EGES_E_NULLPTR, "NULL argument");
  if (signer < 0 || signer > 2) return set_err(EGES_E_INVALID_ARG, "bad signer %d", signer);
  HostJob j;
  j.kind = HostJob::SENDER;
  j.a = sighash;
  j.b = r;
  j.c = s;
  j.d = v;
  j.e = vflags;
  j.signer = signer;
  j.chain_id = chain_id;
  j.addr = addr_out;
  j.status = status;
  return run_host(j, n);
}

int eges_sender_raw_batch(const uint8_t* raw, const uint64_t* offsets, size_t n, int signer, uint64_t chain_id,
                          uint8_t* addr_out, uint8_t* status, uint8_t* sighash_out) {
  if (n == 0) return EGES_SUCCESS;
  if (!offsets || !addr_out || !status) return set_err(EGES_E_NULLPTR, "NULL argument");
  if (signer < 0 || signer > 2) return set_err(EGES_E_INVALID_ARG, "bad signer %d", signer);
  for (size_t i = 0; i < n; ++i)
    if (offsets[i + 1] < offsets[i]) return set_err(EGES_E_INVALID_ARG, "offsets decrease at %zu", i);
  if (!raw && offsets[n] != offsets[0]) return set_err(EGES_E_NULLPTR, "raw is NULL");
  HostJob j;
  j.kind = HostJob::SENDER_RAW;
  j.a = raw;
  j.offsets = offsets;
  j.signer = signer;
  j.chain_id = chain_id;
  j.addr = addr_out;
  j.status = status;
  j.sighash = sighash_out;
  return run_host(j, n);
}

int eges_block_senders_raw(const uint8_t* block, size_t len, uint32_t lists, int signer, uint64_t chain_id,
                           size_t cap, uint8_t* addr_out, uint8_t* status, uint32_t* counts, int* block_status) {
  if (!block || !counts || !block_status) return set_err(EGES_E_NULLPTR, "NULL argument");
  if (signer < 0 || signer > 2) return set_err(EGES_E_INVALID_ARG, "bad signer %d", signer);
  std::vector<uint64_t> offs[3];
  counts[0] = counts[1] = counts[2] = 0;
  if (!split_extblock(block, len, offs)) {
    *block_status = EGES_DECODE_FAILED;
    return EGES_SUCCESS;
  }
  // the structure decodes: counts are valid from here on, also when the selected lists exceed
  // cap (the caller's sizing call, which returns before any transaction is decoded: its
  // *block_status then covers the structure only, include/eges.h)
  *block_status = EGES_OK;
  size_t total = 0;
  for (int k = 0; k < 3; ++k) {
    counts[k] = (uint32_t)(offs[k].size() - 1);
    if (lists & (1u << k)) total += counts[k];
  }
  if (total > cap) return set_err(EGES_E_INVALID_ARG, "block has %zu selected transactions, cap %zu", total, cap);
  if (total && (!addr_out || !status)) return set_err(EGES_E_NULLPTR, "NULL output");
  size_t base = 0;
  for (int k = 0; k < 3; ++k) {
    if (counts[k] == 0) continue;
    const std::vector<uint64_t>& o = offs[k];
    if (!(lists & (1u << k))) {
      // rlp.DecodeBytes(block) decodes every list: an undecodable transaction of an unselected
      // list fails the block too. Decode-only pass (the GPU decoder, no recovery).
      bool bad = false;
      const int rc = decode_check_raw(block + o[0], o.data(), counts[k], signer, chain_id, &bad);
      if (rc) return rc;
      if (bad) *block_status = EGES_DECODE_FAILED;
      continue;
    }
    const int rc = eges_sender_raw_batch(block + o[0], o.data(), counts[k], signer, chain_id, addr_out + base * 20,
                                         status + base, nullptr);
    if (rc) return rc;
    base += counts[k];
  }
  // rlp.DecodeBytes of the block fails on any undecodable transaction of the selected lists
  for (size_t i = 0; i < total; ++i)
    if (status[i] == EGES_DECODE_FAILED) *block_status = EGES_DECODE_FAILED;
  return EGES_SUCCESS;
}

int eges_ecrecover_precompile_batch(const uint8_t* input, const uint32_t* inlen, size_t n, uint8_t* out32,
                                    uint8_t* status) {
  if (n == 0) return EGES_SUCCESS;
  if (!input || !out32 || !status) return set_err(EGES_E_NULLPTR, "NULL argument");
  HostJob j;
  j.kind = HostJob::PRECOMPILE;
  j.a = input;
  j.inlen = inlen;
  j.addr = out32;
  j.status = status;
  return run_host(j, n);
}

int eges_verify_batch(const uint8_t* pub, const uint8_t* publen, const uint8_t* msg, const uint8_t* sig, size_t n,
                      uint8_t* ok_out) {
  if (n == 0) return EGES_SUCCESS;
  if (!pub || !publen || !msg || !sig || !ok_out) return set_err(EGES_E_NULLPTR, "NULL argument");
  HostJob j;
  j.kind = HostJob::VERIFY;
  j.a = pub;
  j.b = publen;
  j.c = msg;
  j.d = sig;
  j.status = ok_out;
  return run_host(j, n);
}

int eges_ecdsa_recover(unsigned char* pubkey_out65, const unsigned char* sigdata65, const unsigned char* msgdata32) {
  if (!pubkey_out65 || !sigdata65 || !msgdata32) return 0;
  RecoverReq r{msgdata32, sigdata65, pubkey_out65};
  g_recover_co.submit(&r);
  // the reference returns 0 for every failure; an engine failure (no device, HIP error) also
  // leaves its text for eges_last_error on this caller's thread, and "" on success
  t_err = r.rc ? r.err : std::string();
  return r.result;
}

int eges_ecdsa_verify(const unsigned char* sigdata64, const unsigned char* msgdata32, const unsigned char* pubkeydata,
                      size_t pubkeylen) {
  if (!sigdata64 || !msgdata32 || !pubkeydata) return 0;
  if (pubkeylen != 33 && pubkeylen != 65) return 0;  // eckey_pubkey_parse accepts only these sizes
  VerifyReq r{sigdata64, msgdata32, pubkeydata, (uint8_t)pubkeylen};
  g_verify_co.submit(&r);
  t_err = r.rc ? r.err : std::string();
  return r.result;
}

int eges_ecrecover_batch_dev(int device, const uint8_t* msg, const uint8_t* sig, size_t n, uint8_t* pub_out,
                             uint8_t* addr_out, uint8_t* status, void* stream) {
  if (n == 0) return EGES_SUCCESS;
  if (!msg || !sig || !status) return set_err(EGES_E_NULLPTR, "NULL argument");
  int rc = ensure_init();
  if (rc) return rc;
  DevPtr d = dev_by_id(device);
  if (!d) return set_err(EGES_E_INVALID_ARG, "device %d not managed by the engine", device);
  DeviceWide wide(*d);
  DevGuard g(device);
  return run_recover_dev(*d, Route::now(), msg, sig, n, pub_out, addr_out, status, (hipStream_t)stream);
}

int eges_sender_batch_dev(int device, const uint8_t* sighash, const uint8_t* r, const uint8_t* s, const uint8_t* v,
                          const uint8_t* vflags, size_t n, int signer, uint64_t chain_id, uint8_t* addr_out,
                          uint8_t* status, void* stream) {
  if (n == 0) return EGES_SUCCESS;
  if (!sighash || !r || !s || !v || !addr_out || !status) return set_err(EGES_E_NULLPTR, "NULL argument");
  if (signer < 0 || signer > 2) return set_err(EGES_E_INVALID_ARG, "bad signer %d", signer);
  int rc = ensure_init();
  if (rc) return rc;
  DevPtr d = dev_by_id(device);
  if (!d) return set_err(EGES_E_INVALID_ARG, "device %d not managed by the engine", device);
  DeviceWide wide(*d);
  DevGuard g(device);
  return run_sender_dev(*d, Route::now(), sighash, r, s, v, vflags, n, signer, chain_id, addr_out, status,
                        (hipStream_t)stream);
}

int eges_sender_raw_batch_dev(int device, const uint8_t* raw, const uint64_t* offsets, size_t n, int signer,
                              uint64_t chain_id, uint8_t* addr_out, uint8_t* status, uint8_t* sighash_out,
                              void* stream) {
  if (n == 0) return EGES_SUCCESS;
  if (!raw || !offsets || !addr_out || !status) return set_err(EGES_E_NULLPTR, "NULL argument");
  if (signer < 0 || signer > 2) return set_err(EGES_E_INVALID_ARG, "bad signer %d", signer);
  int rc = ensure_init();
  if (rc) return rc;
  DevPtr d = dev_by_id(device);
  if (!d) return set_err(EGES_E_INVALID_ARG, "device %d not managed by the engine", device);
  DeviceWide wide(*d);
  DevGuard g(device);
  return run_sender_raw_dev(*d, Route::now(), raw, offsets, n, signer, chain_id, addr_out, status, sighash_out,
                            (hipStream_t)stream);
}

int eges_ecrecover_precompile_batch_dev(int device, const uint8_t* input, const uint32_t* inlen, size_t n,
                                        uint8_t* out32, uint8_t* status, void* stream) {
  if (n == 0) return EGES_SUCCESS;
  if (!input || !out32 || !status) return set_err(EGES_E_NULLPTR, "NULL argument");
  int rc = ensure_init();
  if (rc) return rc;
  DevPtr d = dev_by_id(device);
  if (!d) return set_err(EGES_E_INVALID_ARG, "device %d not managed by the engine", device);
  DeviceWide wide(*d);
  DevGuard g(device);
  return run_precompile_dev(*d, Route::now(), input, inlen, n, out32, status, (hipStream_t)stream);
}

int eges_verify_batch_dev(int device, const uint8_t* pub, const uint8_t* publen, const uint8_t* msg, const uint8_t* sig,
                          size_t n, uint8_t* ok_out, void* stream) {
  if (n == 0) return EGES_SUCCESS;
  if (!pub || !publen || !msg || !sig || !ok_out) return set_err(EGES_E_NULLPTR, "NULL argument");
  int rc = ensure_init();
  if (rc) return rc;
  DevPtr d = dev_by_id(device);
  if (!d) return set_err(EGES_E_INVALID_ARG, "device %d not managed by the engine", device);
  DeviceWide wide(*d);
  DevGuard g(device);
  return run_verify_dev(*d, Route::now(), pub, publen, msg, sig, n, ok_out, (hipStream_t)stream);
}

static int synth_common(int device, uint64_t first_index, size_t n, const uint8_t* msg_in, uint8_t* msg, uint8_t* sig,
                        uint8_t* addr_expected, void* stream) {
  int rc = ensure_init();
  if (rc) return rc;
  DevPtr d = dev_by_id(device);
  if (!d) return set_err(EGES_E_INVALID_ARG, "device %d not managed by the engine", device);
  DeviceWide wide(*d);
  DevGuard g(device);
  hipStream_t st = (hipStream_t)stream;
  Serial ser(*d, st);
  for (size_t off = 0; off < n; off += CHUNK) {
    const uint32_t m = (uint32_t)std::min(CHUNK, n - off);
    SynthParams p{first_index + off, m, msg_in ? msg_in + off * 32 : nullptr, msg ? msg + off * 32 : nullptr,
                  sig + off * 65, addr_expected + off * 20, d->gtab, d->ws};
    HIPCHK(launch_synth(p, d->mb_synth, st));
  }
  return EGES_SUCCESS;
}

int eges_synth_sign_dev(int device, uint64_t first_index, size_t n, uint8_t* msg, uint8_t* sig, uint8_t* addr_expected,
                        void* stream) {
  if (n == 0) return EGES_SUCCESS;
  if (!msg || !sig || !addr_expected) return set_err(EGES_E_NULLPTR, "NULL argument");
  return synth_common(device, first_index, n, nullptr, msg, sig, addr_expected, stream);
}

int eges_synth_sign_msg_dev(int device, uint64_t first_index, size_t n, const uint8_t* msg_in, uint8_t* sig,
                            uint8_t* addr_expected, void* stream) {
  if (n == 0) return EGES_SUCCESS;
  if (!msg_in || !sig || !addr_expected) return set_err(EGES_E_NULLPTR, "NULL argument");
  return synth_common(device, first_index, n, msg_in, nullptr, sig, addr_expected, stream);
}

int eges_diag_counters(int device, uint64_t* out, size_t n, int reset) {
  if (!out && n) return set_err(EGES_E_NULLPTR, "out is NULL");
  std::vector<DevPtr> devs;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    for (const DevPtr& d : g_devs)
      if (d->id == device) devs.push_back(d);
  }
  if (devs.empty()) return set_err(EGES_E_INVALID_ARG, "device %d not managed by the engine", device);
  uint64_t sum[DIAG_WORDS] = {0};
  for (const DevPtr& d : devs) {  // every logical instance of the device
    std::lock_guard<std::mutex> dl(d->mu);
    DevGuard g(d->id);
    uint32_t w[DIAG_WORDS];
    HIPCHK(hipDeviceSynchronize());  // the lanes' and the callers' streams too
    HIPCHK(hipMemcpy(w, d->diag, sizeof w, hipMemcpyDeviceToHost));
    for (int k = 0; k < DIAG_WORDS; ++k) sum[k] += w[k];
    if (reset) HIPCHK(hipMemset(d->diag, 0, sizeof w));
  }
  for (size_t k = 0; k < n && k < (size_t)DIAG_WORDS; ++k) out[k] = sum[k];
  return EGES_SUCCESS;
}

int eges_test_set_knob(const char* name, long long value) {
  knobs_load_env();  // a value set before the first eges_init is not overwritten by it
  const int k = knob_index(name);
  if (k < 0) return set_err(EGES_E_INVALID_ARG, "unknown knob %s", name ? name : "(null)");
  g_knob[k].store(value, std::memory_order_relaxed);
  return EGES_SUCCESS;
}

int eges_test_get_knob(const char* name, long long* value) {
  knobs_load_env();
  const int k = knob_index(name);
  if (k < 0) return set_err(EGES_E_INVALID_ARG, "unknown knob %s", name ? name : "(null)");
  if (!value) return set_err(EGES_E_NULLPTR, "value is NULL");
  *value = g_knob[k].load(std::memory_order_relaxed);
  return EGES_SUCCESS;
}

void eges_keccak256(const uint8_t* data, size_t len, uint8_t* out32) {
  uint64_t st[25] = {0};
  const size_t rate = 136;
  while (len >= rate) {
    for (size_t i = 0; i < rate / 8; ++i) {
      uint64_t w = 0;
      for (int b = 0; b < 8; ++b) w |= (uint64_t)data[8 * i + b] << (8 * b);
      st[i] ^= w;
    }
    keccakf_host(st);
    data += rate;
    len -= rate;
  }
  uint8_t blk[136] = {0};
  if (len) std::memcpy(blk, data, len);
  blk[len] ^= 0x01;
  blk[rate - 1] ^= 0x80;
  for (size_t i = 0; i < rate / 8; ++i) {
    uint64_t w = 0;
    for (int b = 0; b < 8; ++b) w |= (uint64_t)blk[8 * i + b] << (8 * b);
    st[i] ^= w;
  }
  keccakf_host(st);
  for (int i = 0; i < 32; ++i) out32[i] = (uint8_t)(st[i / 8] >> (8 * (i % 8)));
}

}  // extern "C"
