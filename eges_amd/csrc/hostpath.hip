// Host-buffer paths (engine.h): the chunked pipeline, the multi-device split, the Geec block split
// and the host Keccak.
#include "engine.h"

namespace eges::host {

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
// ------------------------------------------------------------------ host-buffer pipelines

// Device bytes of one pipeline region for a chunk of m items: inputs | scratch | outputs.
struct Region {
  size_t in_bytes = 0, raw_lo = 0, raw_len = 0, o_rec = 0, o_out = 0, total = 0;
};
// Every input array of a region starts on a 128-byte line (LINE): a gated call opens its inputs
// piece by piece, and no line may hold bytes of two arrays, one of which a workgroup reads before
// the piece holding the other's bytes is open (that line would then sit in L2 with stale bytes).
constexpr size_t LINE = 128;
Region region_for(const HostJob& j, size_t base, size_t m) {
  Region g;
  const size_t m_pad = align_up(m, 64);
  const size_t a32 = align_up(m * 32, LINE);
  switch (j.kind) {
    case HostJob::RECOVER: g.in_bytes = a32 + align_up(m * 65, LINE); break;
    case HostJob::SENDER: g.in_bytes = 4 * a32 + align_up(m, LINE); break;
    case HostJob::VERIFY: g.in_bytes = align_up(m * 65, LINE) + align_up(m, LINE) + a32 + align_up(m * 64, LINE); break;
    case HostJob::PRECOMPILE: g.in_bytes = align_up(m * 128, LINE) + align_up(m * 4, LINE); break;
    case HostJob::SENDER_RAW:
      g.raw_lo = j.offsets[base] - j.offsets[0];
      g.raw_len = j.offsets[base + m] - j.offsets[base];
      g.in_bytes = align_up(g.raw_len, LINE) + align_up(8 * (m + 1), LINE) + tx_rows_bytes(m);
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
  // The deferred copies of a gated chunk, opened in pieces of `per` items in item order (the
  // mid-size kernels' workgroup order): each queued array knows its item stride (0: the wire bytes,
  // cut at the offsets; -1: the offsets array itself, n + 1 entries) so a piece copies only its
  // items' bytes, then publishes base + piece + 1 (handoff.cuh gate_wait).
  struct GateOpen {
    struct Copy {
      uint8_t* dst;
      const uint8_t* src;
      size_t n;
      long stride;
    } q[8];
    int nq = 0;
    const uint64_t* offs = nullptr;  // the wire form's host offsets of this chunk (stride 0)
    size_t items = 0, per = 0;
    uint32_t* w = nullptr;  // armed: the kernels wait for sequence `seq` (the last piece)
    uint32_t seq = 0, pieces = 1;
    void copy_range(const Copy& c, size_t lo, size_t hi) const {
      size_t a, b;
      if (c.stride > 0) {
        a = lo * (size_t)c.stride;
        b = hi * (size_t)c.stride;
      } else if (c.stride == 0) {
        a = offs[lo] - offs[0];
        b = offs[hi] - offs[0];
      } else {  // entries lo .. hi: item hi - 1 ends at entry hi (the next piece copies it again)
        a = lo * 8;
        b = (hi + 1) * 8;
      }
      // (to the end of the line the piece's last bytes, and a dword read past them, fall in: a
      // workgroup of this piece may bring that line into L2, so it must hold the next piece's
      // first bytes already; they are the same bytes, copied again with that piece)
      b = std::min(c.n, align_up(b + 4, LINE));
      if (b > a) std::memcpy(c.dst + a, c.src + a, b - a);
    }
    void open() {
      if (nq) {
        const size_t step = pieces > 1 ? per : items;
        for (uint32_t p = 0; p < pieces; ++p) {
          const size_t lo = (size_t)p * step, hi = std::min(items, lo + step);
          for (int i = 0; i < nq; ++i) copy_range(q[i], lo, hi);
          if (w) publish_u32(w, seq - pieces + p + 1);
        }
      }
      nq = 0;
      if (w) publish_u32(w, seq);
      w = nullptr;
    }
    ~GateOpen() { open(); }
  } gopen;
  bool defer = false;  // this chunk's inputs wait for gopen.open()
  auto arm = [&](RecoverParams& p) {  // a deferred chunk's kernels wait at the gate
    if (!defer || p.n == 0) return;
    // pieces of GATE_STEP workgroups (64 items each) when the grid has several of them
    const uint32_t wgs = (p.n + MID_SIGS_PER_BLOCK - 1) / MID_SIGS_PER_BLOCK;
    const uint32_t step = rt.gate_step > 0 ? (uint32_t)rt.gate_step : wgs;
    const uint32_t pieces = (wgs + step - 1) / step;
    gate.seq += pieces;  // (wraps harmlessly: every comparison is a sequence difference)
    p.gate = gate.w;
    p.gate_dev = gate.dev;
    p.gate_seq = gate.seq;
    p.gate_step = pieces > 1 ? step : 0u;
    p.gate_pieces = pieces;
    gopen.w = gate.w;
    gopen.seq = gate.seq;
    gopen.pieces = pieces;
    gopen.items = p.n;
    gopen.per = (size_t)step * MID_SIGS_PER_BLOCK;
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
  auto h2d = [&](uint8_t* B, uint8_t* dst, const void* src, size_t bytes, long stride) -> int {
    if (!bytes) return EGES_SUCCESS;
    if (pinned) {  // dst points into the pinned buffer (see I below)
      if (defer && gopen.nq < 8) gopen.q[gopen.nq++] = {dst, static_cast<const uint8_t*>(src), bytes, stride};
      else std::memcpy(dst, src, bytes);  // (at most 5 inputs per kind: q never fills)
      return EGES_SUCCESS;
    }
    (void)B;
    HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, sx));
    return EGES_SUCCESS;
  };
  auto flush_in = [&](uint8_t*) -> int { return EGES_SUCCESS; };
#define H2D(B, dst, src, bytes, stride)                   \
  do {                                                     \
    int rc_ = h2d((B), (dst), (src), (bytes), (stride));   \
    if (rc_) return rc_;                                   \
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
  auto sighash_off = [&](const Pending& q) { return align_up(q.g.raw_len, LINE) + align_up(8 * (q.m + 1), LINE); };
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
      uint8_t* ds = dm + align_up(m * 32, LINE);
      const bool fused = fused_parse(d, rt, m);
      defer = gating && fused && use_mid(d, rt, m);  // (the latency kernels measured +-0 to +1.5 % slower)
      H2D(B, dm, j.a + base * 32, m * 32, 32);
      H2D(B, ds, j.b + base * 65, m * 65, 65);
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
      HIPCHK(launch_recover_pass(d, rt, p, sk, rt.host_gens));
    } else if (j.kind == HostJob::SENDER) {
      const size_t a32 = align_up(m * 32, LINE);
      uint8_t* dh = I;
      uint8_t* dr = dh + a32;
      uint8_t* dsv = dr + a32;
      uint8_t* dv = dsv + a32;
      uint8_t* df = dv + a32;
      const bool fused = sender_fused(d, rt, m, {dh, dr, dsv, dv});
      defer = gating && fused && use_mid(d, rt, m);  // (the latency kernels measured +-0 to +1.5 % slower)
      H2D(B, dh, j.a + base * 32, m * 32, 32);
      H2D(B, dr, j.b + base * 32, m * 32, 32);
      H2D(B, dsv, j.c + base * 32, m * 32, 32);
      H2D(B, dv, j.d + base * 32, m * 32, 32);
      if (j.e) H2D(B, df, j.e + base, m, 1);
      FLUSH_IN(B);
      JOIN_IN(r);
      RecoverParams p{rec, (uint32_t)m, (uint32_t)m_pad, o_st, o_addr, nullptr, d.gtab, wsk};
      if (fused)  // the recover kernel reads the rows itself
        bind_sender_rows(p, dh, dr, dsv, dv, j.e ? df : nullptr, j.signer, j.chain_id);
      else
        HIPCHK(launch_prep_sender(dh, dr, dsv, dv, j.e ? df : nullptr, (uint32_t)m, (uint32_t)m_pad, j.signer, j.chain_id,
                                  rec, sk));
      arm(p);
      HIPCHK(launch_recover_pass(d, rt, p, sk, rt.host_gens));
    } else if (j.kind == HostJob::PRECOMPILE) {
      uint8_t* din = I;
      uint32_t* dlen = reinterpret_cast<uint32_t*>(din + align_up(m * 128, LINE));
      H2D(B, din, j.a + base * 128, m * 128, 128);
      if (j.inlen) H2D(B, reinterpret_cast<uint8_t*>(dlen), j.inlen + base, m * 4, 4);
      FLUSH_IN(B);
      JOIN_IN(r);
      if (pinned) std::memset(o_addr, 0, m * 32);
      else HIPCHK(hipMemsetAsync(o_addr, 0, m * 32, sk));
      HIPCHK(launch_prep_precompile(din, j.inlen ? dlen : nullptr, (uint32_t)m, (uint32_t)m_pad, rec, sk));
      RecoverParams p{rec, (uint32_t)m, (uint32_t)m_pad, o_st, o_addr + 12, nullptr, d.gtab, wsk, 32};
      HIPCHK(launch_recover_pass(d, rt, p, sk, rt.host_gens));
    } else if (j.kind == HostJob::SENDER_RAW) {
      uint8_t* draw = I;
      uint64_t* doff = reinterpret_cast<uint64_t*>(draw + align_up(rg.raw_len, LINE));
      uint8_t* hs = B + align_up(rg.raw_len, LINE) + align_up(8 * (m + 1), LINE);  // decoded rows: device memory
      uint8_t* rr = hs + m * 32;
      uint8_t* sr = rr + m * 32;
      uint8_t* vr = sr + m * 32;
      uint8_t* vf = vr + m * 32;
      // (the fused form reads the encodings straight from the pinned buffer: a pipelined host copy
      // + DMA into device memory measured 0.486-0.508 ms against 0.450 ms for C1, same kernel)
      const bool fused = !j.decode_only && wire_fused(d, rt, m, draw);
      defer = gating && fused && use_mid(d, rt, m);  // (the latency kernels measured +-0 to +1.5 % slower)
      if (defer) gopen.offs = j.offsets + base;  // (the raw bytes open at these offsets, piece by piece)
      if (rg.raw_len) H2D(B, draw, j.a + rg.raw_lo, rg.raw_len, 0);
      H2D(B, reinterpret_cast<uint8_t*>(doff), j.offsets + base, 8 * (m + 1), -1);
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
        HIPCHK(launch_recover_pass(d, rt, p, sk, rt.host_gens));
      }
    } else {
      uint8_t* dp = I;
      uint8_t* dl = dp + align_up(m * 65, LINE);
      uint8_t* dm = dl + align_up(m, LINE);
      uint8_t* ds = dm + align_up(m * 32, LINE);
      H2D(B, dp, j.a + base * 65, m * 65, 65);
      H2D(B, dl, j.b + base, m, 1);
      H2D(B, dm, j.c + base * 32, m * 32, 32);
      H2D(B, ds, j.d + base * 64, m * 64, 64);
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
  // every output is read after the streams' completion signal (handoff.cuh: an in-kernel flag
  // word can reach the host before the outputs stored ahead of it)
  HIPCHK(hipStreamSynchronize(sx));
  if (sx != st) HIPCHK(hipStreamSynchronize(st));  // (st's last work is already behind sx's events)
  HSTAMP(4);
  drain.armed = false;
  if (gating && __atomic_load_n(&gate.w[1], __ATOMIC_ACQUIRE) != 0u) {
    __atomic_store_n(&gate.w[1], 0u, __ATOMIC_RELAXED);
    return set_err(EGES_E_HIP, "a kernel's input gate timed out");
  }
  if (pinned && have_prev) unpack(prev);
  HSTAMP(5);
  if (rt.recheck && pinned && have_prev) {  // tests: did any returned byte change after it was read?
    HIPCHK(hipStreamSynchronize(st));
    const uint8_t* o_pub = pin + prev.g.o_out;
    const uint8_t* o_addr = o_pub + prev.m * 65;
    const uint8_t* o_st = o_addr + prev.m * 32;
    size_t changed = 0;
    for (size_t i = 0; i < prev.m; ++i) {
      const size_t q = prev.base + i;
      const bool same = (!j.status || j.status[q] == o_st[i]) &&
                        (!j.addr || std::memcmp(j.addr + q * astride, o_addr + i * astride, astride) == 0) &&
                        (!j.pub || std::memcmp(j.pub + q * 65, o_pub + i * 65, 65) == 0);
      changed += same ? 0 : 1;
    }
    if (changed) return set_err(EGES_E_HIP, "recheck: %zu items of the pinned outputs changed after the call read them", changed);
  }
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

}  // namespace eges::host
