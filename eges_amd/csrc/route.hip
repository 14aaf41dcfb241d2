// Routing of a call to the kernel forms (latency / mid-size / lane-serial) and the
// device-resident pipelines behind the *_dev entries (engine.h).
#include "engine.h"

namespace eges::host {

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

// batches (or chunks) the mid-size kernel takes: above LAT_MAX, up to MID_MAX and what the
// device workspace holds
// The bucket form (k_recover_mid.hip) holds 152 KB of LDS: one workgroup per CU. It is the
// faster form while the grid fits one generation (n <= 64 x CUs); beyond that the windowed form
// (two workgroups per CU) is (tools/formcurve.py).
bool mid_bucket(const Dev& d, const Route& rt, size_t n) {
  const long long f = rt.mid_form;
  if (f == 0) return false;
  if (f >= 2) return true;
  return (n + MID_SIGS_PER_BLOCK - 1) / MID_SIGS_PER_BLOCK <= (size_t)d.cus;
}
// The bucket form at two workgroups per CU (k_recover_mid.hip G2: its ring and parts in the
// workspace, ~76 KB of LDS, 215 registers): every non-wire bucket-band batch up to one generation
// at two per CU (round 6). Past one generation of the one-per-CU form it
// replaces the windowed form / a second bucket generation (16,385-32,768 signatures 0.70 -> 0.51-
// 0.54 ms, verify 0.64 -> 0.50-0.52 ms); below it, it is also 1-3 % (recovery) and 3-6 % (verify)
// faster than the one-per-CU kernel (profiles/r06/formcurve_b2_*). Wire-format batches whose
// decode is fused in keep the one-per-CU form (its LDS stage); past 64 x CUs they take the
// unfused rows (wire_fused()). EGES_MID_FORM = 2 (tests) keeps the one-per-CU form unless
// EGES_BKT2 = 2.
bool mid_bkt2(const Dev& d, const Route& rt, size_t n) {
  if (rt.bkt2 == 0 || rt.mid_form == 0) return false;
  const size_t wgs = (n + MID_SIGS_PER_BLOCK - 1) / MID_SIGS_PER_BLOCK;
  if (wgs * bkt2_ws_bytes_per_block() > dev_ws_bytes(d)) return false;
  if (rt.bkt2 >= 2) return true;
  return rt.mid_form == 1 && wgs <= 2 * (size_t)d.cus;
}
bool use_mid(const Dev& d, const Route& rt, size_t n) {
  if (n <= rt.lat_max || n > rt.mid_max) return false;
  if (mid_bucket(d, rt, n) || mid_bkt2(d, rt, n)) return true;
  // the windowed form: in auto mode only while its grid is one generation (two workgroups per
  // CU); a second, partial one costs more than the lane-serial kernel's one chain (36k-40k
  // signatures 0.98 against 0.80 ms, profiles/r05/formcurve_cut_r05_zb.jsonl)
  const size_t wgs = (n + MID_SIGS_PER_BLOCK - 1) / MID_SIGS_PER_BLOCK;
  if (rt.mid_form == 1 && wgs > 2 * (size_t)d.cus) return false;
  return wgs * mid_ws_bytes_per_block() <= dev_ws_bytes(d);
}
// VerifySignature batches above LAT_MAX that the bucket form's verify mode takes (EGES_VERIFY_MID_GENS
// generations of workgroups: n <= 64 x CUs x gens), instead of the lane-serial verify kernel's fixed
// chain (one generation 0.35 ms, two 0.66 ms, the lane-serial kernel 0.78-0.82 ms up to 65k items)
bool verify_mid(const Dev& d, const Route& rt, size_t n) {
  return rt.mid_form != 0 && n > rt.lat_max && n <= rt.mid_max &&
         ((n + MID_SIGS_PER_BLOCK - 1) / MID_SIGS_PER_BLOCK <= (size_t)d.cus * (size_t)rt.verify_mid_gens ||
          mid_bkt2(d, rt, n));
}
hipError_t launch_verify_any(Dev& d, const Route& rt, const VerifyParams& p, bool small, hipStream_t st) {
  if (small || p.n <= rt.lat_max) return launch_verify_lat(p, p.n <= rt.wide_max, st);
  if (verify_mid(d, rt, p.n)) return launch_verify_mid(p, p.ws != nullptr && mid_bkt2(d, rt, p.n), dev_ws_bytes(d), st);
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

hipError_t launch_recover_pass(Dev& d, const Route& rt, const RecoverParams& p0, hipStream_t st, int gens) {
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
  if (p.gate && !mid) return hipErrorInvalidValue;  // (only the mid-size kernels wait at the gate)
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
  if (mid && !p.wire_raw && p.ws && mid_bkt2(d, rt, p.n)) return launch_recover_bkt2(p, dev_ws_bytes(d), st);
  if (mid) return launch_recover_mid(p, mid_bucket(d, rt, p.n), dev_ws_bytes(d), st);
  if (p.n <= rt.lat_max || p.raw_sig) return launch_recover_lat(p, st);
  // (EGES_HOST_GENS above the device's EGES_GRID_MULT is clamped to it: the workspace holds
  // ws_blocks, sized for d.gm generations, and a larger grid would be refused)
  const int mb = gens > 0 ? std::max(1, d.mb_recover / d.gm * std::min(gens, d.gm)) : d.mb_recover;
  return launch_recover(p, mb, d.ws_blocks, st);
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

}  // namespace eges::host
