// The single-item seam (eges_ecdsa_recover / eges_ecdsa_verify, engine.h): concurrent callers
// coalesced into shared groups, served by the resident single-call server or a small-call lane.
#include "engine.h"

namespace eges::host {

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

// One job on the resident server of device d: fill(data, layout) writes the inputs, read(data,
// layout) takes the outputs, both at the offsets of the running server's own capacity (r.cap,
// which the kernel was launched with: it changes only while no server runs), never the knob's. Returns -1 when the server is off, busy or the group too large (the caller
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
  const long long idle_us = std::max<long long>(50, knob(KNOB_RESIDENT_IDLE_US));
  const auto now = std::chrono::steady_clock::now();
  // a server idle for half its bound may be deciding to exit: restart it rather than race it
  if (r.running &&
      (hipStreamQuery(r.stream) == hipSuccess || now - r.last_use > std::chrono::microseconds(idle_us / 2)))
    resident_halt(d, r);
  auto launch = [&]() -> int {
    if (!r.running) {  // the lane finishes what it runs and takes no more calls
      std::lock_guard<std::mutex> l0(d.lanes[r.lane].mu);
      d.lanes[r.lane].reserved.store(true, std::memory_order_release);
    }
    HIPCHK(hipMemsetAsync(r.counter, 0, RESIDENT_COUNTER_BYTES, r.stream));
    if (++r.inst == 0) r.inst = 1;
    ResidentParams rp{r.job, r.data, r.cap, __atomic_load_n(&r.job->done, __ATOMIC_ACQUIRE), r.counter,
                      (uint64_t)idle_us * 100ull, r.inst, d.gtab, d.diag};  // (s_memrealtime: 100 MHz)
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
  const ResidentLayout L = resident_layout(r.cap);
  fill(r.data, L);
  __atomic_store_n(&r.job->n, (uint32_t)n, __ATOMIC_RELAXED);
  __atomic_store_n(&r.job->kind, (uint32_t)kind, __ATOMIC_RELAXED);
  const uint32_t seq = ++r.seq;
  publish_u32(&r.job->seq, seq);
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
  // the outputs count only once every item's tag matches the bytes read (launch.h out_tag_*: the
  // done word can reach this thread before the outputs do); a faulted verify item says so in its tag
  bool tag_fault = false;
  for (uint64_t spins = 0;; ++spins) {
    size_t bad = 0;
    tag_fault = false;
    for (size_t i = 0; i < n; ++i) {
      const uint64_t t = __atomic_load_n(reinterpret_cast<const uint64_t*>(r.data + L.tag) + i, __ATOMIC_ACQUIRE);
      if (kind == RESIDENT_RECOVER) {
        const uint8_t* pb = r.data + L.pub + i * 65;
        uint32_t be[16];
        for (int w = 0; w < 16; ++w)
          be[w] = (uint32_t)pb[1 + 4 * w] << 24 | (uint32_t)pb[2 + 4 * w] << 16 | (uint32_t)pb[3 + 4 * w] << 8 | pb[4 + 4 * w];
        bad += t != out_tag_recover(seq, r.data[L.status + i], pb[0], be);
      } else {
        const uint32_t ok = r.data[L.vok + i];
        if (t == out_tag_verify(seq, ok, 1u)) tag_fault = true;
        else bad += t != out_tag_verify(seq, ok, 0u);
      }
    }
    if (bad == 0) break;
    if ((spins & 255) == 255 && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) {
      resident_halt(d, r);
      return set_err(EGES_E_HIP, "resident server: %zu outputs of job %u never matched their tags", bad, seq);
    }
    cpu_relax();
  }
  if (tag_fault) __atomic_store_n(reinterpret_cast<uint32_t*>(r.data + L.vfault), 1u, __ATOMIC_RELAXED);
  if (knob(KNOB_TEST_RECHECK) == 0) {
    read(r.data, L);
    r.last_use = std::chrono::steady_clock::now();
    return EGES_SUCCESS;
  }
  // tests: the call returns what a snapshot taken at the done word holds; 200 us later the live
  // outputs must still be the same bytes
  std::vector<uint8_t> snap(r.data, r.data + L.total);
  read(snap.data(), L);
  r.last_use = std::chrono::steady_clock::now();
  const auto w0 = std::chrono::steady_clock::now();
  while (std::chrono::steady_clock::now() - w0 < std::chrono::microseconds(200)) cpu_relax();
  const bool rec = kind == RESIDENT_RECOVER;
  const size_t a0 = rec ? L.pub : L.vok, a1 = rec ? L.pub + n * 65 : L.vok + n;
  const size_t b0 = rec ? L.status : L.vfault, b1 = rec ? L.status + n : L.vfault + 4;
  if (std::memcmp(snap.data() + a0, r.data + a0, a1 - a0) != 0 || std::memcmp(snap.data() + b0, r.data + b0, b1 - b0) != 0)
    return set_err(EGES_E_HIP, "recheck: the resident server's outputs changed after the call read them (job %u)", seq);
  return EGES_SUCCESS;
}

void run_group(std::vector<RecoverReq*>& g) {
  const size_t n = g.size();
  if (ensure_init() == EGES_SUCCESS) {
    if (DevPtr d = first_dev()) {
      const int rc = resident_job(
          *d, d->res, RESIDENT_RECOVER, n,
          [&](uint8_t* D, const ResidentLayout& L) {
            for (size_t i = 0; i < n; ++i) {
              std::memcpy(D + L.msg + i * 32, g[i]->msg, 32);
              std::memcpy(D + L.sig + i * 65, g[i]->sig, 65);
            }
          },
          [&](const uint8_t* D, const ResidentLayout& L) {
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
      const int rc = resident_job(
          *d, d->res, RESIDENT_VERIFY, n,
          [&](uint8_t* D, const ResidentLayout& L) {
            *reinterpret_cast<uint32_t*>(D + L.vfault) = 0u;
            for (size_t i = 0; i < n; ++i) {
              std::memset(D + L.vpub + i * 65, 0, 65);
              std::memcpy(D + L.vpub + i * 65, g[i]->pub, g[i]->publen);
              D[L.vpublen + i] = g[i]->publen;
              std::memcpy(D + L.vmsg + i * 32, g[i]->msg, 32);
              std::memcpy(D + L.vsig + i * 64, g[i]->sig, 64);
            }
          },
          [&](const uint8_t* D, const ResidentLayout& L) {
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


int single_recover(unsigned char* pub65, const unsigned char* sig65, const unsigned char* msg32) {
  RecoverReq r{msg32, sig65, pub65};
  g_recover_co.submit(&r);
  // the reference returns 0 for every failure; an engine failure (no device, HIP error) also
  // leaves its text for eges_last_error on this caller's thread, and "" on success
  t_err = r.rc ? r.err : std::string();
  return r.result;
}

int single_verify(const unsigned char* sig64, const unsigned char* msg32, const unsigned char* pub, size_t publen) {
  VerifyReq r{sig64, msg32, pub, (uint8_t)publen};
  g_verify_co.submit(&r);
  t_err = r.rc ? r.err : std::string();
  return r.result;
}

}  // namespace eges::host
