// Host engine: the device registry and each device's resources, the knobs (knobs.h), the error
// text and the small helpers every host path uses (engine.h).
#include "engine.h"

namespace eges::host {

thread_local std::string t_err;

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
static const KnobDef KNOB_DEFS[] = {
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
    {"EGES_RESIDENT_IDLE_US", 500},
    {"EGES_GATE", 1},
    {"EGES_GATE_STEP", 8},
    {"EGES_HOST_GENS", 0},
    {"EGES_VERIFY_MID_GENS", 2},
    {"EGES_BKT2", 1},
    {"EGES_TEST_RECHECK", 0},
};
static_assert(sizeof(KNOB_DEFS) / sizeof(KNOB_DEFS[0]) == KNOB_COUNT, "a name and default for every knob");
std::atomic<long long> g_knob[KNOB_COUNT];
static std::once_flag g_knob_once;

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

std::mutex g_mu;
std::vector<DevPtr> g_devs;
bool g_inited = false;

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
  d->gm = gm;
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

DevPtr first_dev() {
  std::lock_guard<std::mutex> lk(g_mu);
  return g_devs.empty() ? nullptr : g_devs[0];
}

size_t dev_ws_bytes(const Dev& d) { return ws_bytes_per_block() * (size_t)d.ws_blocks; }

}  // namespace eges::host

namespace eges {
long long knob(KnobId k) { return host::g_knob[k].load(std::memory_order_relaxed); }
}  // namespace eges
