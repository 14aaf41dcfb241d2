"""Phase breakdown of the latency kernel on a C3 block (1000 EIP-155 transactions, 100-byte payload):
sender rows (eges_sender_batch) against wire bytes (eges_sender_raw_batch, the fused decode and
signing hash), through the diagnostic build libeges_diag.so (k_recover_lat.hip stamps: wave 0's
phases, wave 1's r^-1 and digits in slots 2 / 7).

Usage: python tools/phases_lat_wire.py [n]
"""
import ctypes
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from eges_amd import _lib, txs  # noqa: E402

lib = ctypes.CDLL(os.path.join(ROOT, "eges_amd", os.environ.get("EGES_DIAG_LIB", "libeges_diag.so")))
for name, (res, args) in _lib.SIGNATURES.items():
    f = getattr(lib, name)
    f.restype, f.argtypes = res, args
lib.eges_diag_read_stamps.restype = ctypes.c_size_t
lib.eges_diag_read_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
PHASES = ["parse + x, c", "wait: wave 1 r^-1+digits", "(wave 1: r^-1)", "R' table", "Strauss + join",
          "Z^-1+affine", "keccak+store", "(wave 1: u1,u2,GLV,digits)"]

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
assert lib.eges_init(0, 0) == 0
dev = torch.device("cuda:0")
sighash = txs.geec_block(0, n, payload=100)
msg = torch.from_numpy(np.ascontiguousarray(sighash)).to(dev)
sig = torch.empty((n, 65), dtype=torch.uint8, device=dev)
exp = torch.empty((n, 20), dtype=torch.uint8, device=dev)
torch.cuda.synchronize()
assert lib.eges_synth_sign_msg_dev(0, 0, n, msg.data_ptr(), sig.data_ptr(), exp.data_ptr(), None) == 0, \
    lib.eges_last_error()
torch.cuda.synchronize()
sig_h, exp_h = sig.cpu().numpy(), exp.cpu().numpy()
r, s, v = (np.ascontiguousarray(x) for x in txs.sender_rows(sig_h, txs.GEEC_CHAIN_ID))
sighash = np.ascontiguousarray(sighash)
raws = txs.geec_block_raw(0, sig_h, payload=100)
offs = np.zeros(n + 1, np.uint64)
offs[1:] = np.cumsum([len(x) for x in raws])
raw = np.frombuffer(b"".join(raws), np.uint8).copy()
P = lambda a: ctypes.c_void_p(a.ctypes.data)  # noqa: E731
T = lambda a: ctypes.c_void_p(a.data_ptr())  # noqa: E731
dv = {k: torch.from_numpy(x).to(dev) for k, x in (("h", sighash), ("r", r), ("s", s), ("v", v), ("f", np.zeros(n, np.uint8)),
                                                  ("raw", raw), ("off", offs.astype(np.int64)))}
ad = torch.empty((n, 20), dtype=torch.uint8, device=dev)
sd = torch.empty(n, dtype=torch.uint8, device=dev)
addr = np.zeros((n, 20), np.uint8)
st = np.zeros(n, np.uint8)
vf = np.zeros(n, np.uint8)
for mode in ("rows", "rows_dev", "wire", "wire_dev"):
    for it in range(3):
        addr.fill(0)
        t0 = time.perf_counter()
        if mode == "wire":
            rc = lib.eges_sender_raw_batch(P(raw), P(offs), n, _lib.SIGNER_EIP155, txs.GEEC_CHAIN_ID, P(addr), P(st), None)
        elif mode == "rows_dev":
            rc = lib.eges_sender_batch_dev(0, T(dv["h"]), T(dv["r"]), T(dv["s"]), T(dv["v"]), T(dv["f"]), n,
                                           _lib.SIGNER_EIP155, txs.GEEC_CHAIN_ID, T(ad), T(sd), None)
        elif mode == "wire_dev":
            rc = lib.eges_sender_raw_batch_dev(0, T(dv["raw"]), T(dv["off"]), n, _lib.SIGNER_EIP155, txs.GEEC_CHAIN_ID,
                                               T(ad), T(sd), None, None)
        else:
            rc = lib.eges_sender_batch(P(sighash), P(r), P(s), P(v), P(vf), n, _lib.SIGNER_EIP155, txs.GEEC_CHAIN_ID,
                                       P(addr), P(st))
        assert rc == 0, lib.eges_last_error()
        if mode.endswith("_dev"):
            torch.cuda.synchronize()
            addr[:] = ad.cpu().numpy()
            st[:] = sd.cpu().numpy()
        dt = time.perf_counter() - t0
    assert np.array_equal(addr, exp_h) and int(st.max()) == 0, mode
    waves = lib.eges_diag_read_stamps(None, 1 << 30)
    buf = (ctypes.c_uint64 * (waves * 8))()
    lib.eges_diag_read_stamps(buf, waves)
    a = np.frombuffer(buf, dtype=np.uint64).reshape(waves, 8).copy()
    a[:, [2, 7]] &= np.uint64(0xFFFFFFFF)
    a = a.astype(np.float64)
    tot = a.sum(axis=1) - a[:, 2] - a[:, 7]
    print(f"{mode}: n={n} call {dt * 1e3:.3f} ms (stamped build), waves={waves}")
    print(f"  per-wave total: mean {tot.mean():.4g} min {tot.min():.4g} max {tot.max():.4g} (s_memtime ticks)")
    for i in range(8):
        m = a[:, i].mean()
        print(f"  {PHASES[i]:28s} {m:12.4g} ticks/wave  {100 * m / tot.mean():5.1f}%")
