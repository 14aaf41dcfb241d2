// C-ABI of libeges.so (include/eges.h): device management, staging, multi-GPU sharding.
//
// Replaces the reference's cgo seam (crypto/secp256k1/secp256.go:45-134, ext.h:18-75). There is
// no CPU compute path here: every recovery / verification runs on gfx950 through the kernels in
// k_*.hip, and the entries fail with EGES_E_NODEVICE when no such device is usable. The engine
// behind it: engine.hip (devices, knobs), route.hip (kernel forms, device-resident pipelines),
// hostpath.hip (host-buffer paths), single.hip (the single-item seam); engine.h declares them.
#include "engine.h"

using namespace eges::host;

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
  return single_recover(pubkey_out65, sigdata65, msgdata32);
}

int eges_ecdsa_verify(const unsigned char* sigdata64, const unsigned char* msgdata32, const unsigned char* pubkeydata,
                      size_t pubkeylen) {
  if (!sigdata64 || !msgdata32 || !pubkeydata) return 0;
  if (pubkeylen != 33 && pubkeylen != 65) return 0;  // eckey_pubkey_parse accepts only these sizes
  return single_verify(sigdata64, msgdata32, pubkeydata, pubkeylen);
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

int eges_diag_resident_running(int device) {
  std::vector<DevPtr> devs;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    for (const DevPtr& d : g_devs)
      if (d->id == device) devs.push_back(d);
  }
  if (devs.empty()) return set_err(EGES_E_INVALID_ARG, "device %d not managed by the engine", device);
  for (const DevPtr& d : devs) {
    std::unique_lock<std::mutex> lk(d->res.mu, std::try_to_lock);
    if (!lk.owns_lock()) return 1;  // (a job is being handed over right now)
    if (d->res.running && hipStreamQuery(d->res.stream) == hipErrorNotReady) return 1;
  }
  return 0;
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

