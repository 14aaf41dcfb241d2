"""Per-role phase breakdown of the mid-size recover kernel (PHASES_WIRE=1: C1-shaped wire-format
batches through eges_sender_raw_batch, the fused path) (diagnostic build libeges_diag.so,
k_recover_mid.hip stamps: one row of 8 s_memtime tick sums per wave).

Usage: python tools/phases_mid.py [n ...]   (forces the mid-size kernel with engine knobs)
"""
import ctypes
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from eges_amd import _lib  # noqa: E402

lib = ctypes.CDLL(os.path.join(ROOT, "eges_amd", os.environ.get("EGES_DIAG_LIB", "libeges_diag.so")))
for name, (res, args) in _lib.SIGNATURES.items():
    f = getattr(lib, name)
    f.restype, f.argtypes = res, args
lib.eges_diag_read_stamps.restype = ctypes.c_size_t
lib.eges_diag_read_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]

ROLES = {
    0: ("A", {0: "parse + R'", 3: "R' table (16)", 1: "wait: digits", 4: "low windows", 7: "wait: y, high parts",
              2: "joins", 5: "Z^-1 + affine", 6: "Keccak + stores"}),
    1: ("S", {0: "parse", 1: "r^-1, u1, u2", 2: "GLV + digits", 3: "y (sqrt)", 4: "u1 G comb"}),
    2: ("B", {0: "parse + R'", 1: "D = 2^75 R'", 2: "D table (8)", 3: "wait: digits", 4: "high windows"}),
    3: ("C", {0: "parse + R'", 1: "D = 2^75 R'", 2: "D table (8)", 3: "wait: digits", 4: "high windows"}),
}

BUCKET_ROLES = {
    0: ("X", {0: "parse + R'", 1: "126 doublings", 2: "ring waits, B1 + B3 joins"}),
    1: ("S", {0: "parse", 1: "r^-1, u1, u2", 2: "GLV + digits", 5: "sighash (wire)", 3: "y (sqrt)",
              4: "u1 G comb"}),
    2: ("Y1", {0: "parse", 1: "wait: digits", 2: "bucket adds", 3: "wait: P_3k", 4: "bucket sums",
               5: "joins (+ waits)", 6: "Z^-1 + affine", 7: "Keccak + stores"}),
    3: ("Y2", {0: "parse", 1: "wait: digits", 2: "bucket adds", 3: "wait: P_3k", 4: "bucket sums"}),
}
FORM = int(os.environ.get("EGES_MID_FORM", "2"))
if FORM:
    ROLES = BUCKET_ROLES
assert lib.eges_init(0, 0) == 0, lib.eges_last_error()
assert lib.eges_test_set_knob(b"EGES_MID_FORM", FORM) == 0
assert lib.eges_test_set_knob(b"EGES_LAT_MAX", 0) == 0 and lib.eges_test_set_knob(b"EGES_MID_MAX", 1 << 20) == 0
dev = torch.device("cuda:0")
WIRE = os.environ.get("PHASES_WIRE") == "1"  # C1-shaped wire-format batches (the fused path)
if WIRE:
    BUCKET_ROLES[0][1][0] = "stage + wait for x"
    BUCKET_ROLES[2][1][0] = "stage"
    BUCKET_ROLES[3][1][0] = "stage"
    BUCKET_ROLES[1][1][0] = "stage + decode + checks"


def run_wire(n):
    from eges_amd import txs
    h = txs.c1_sighashes(0, n)
    hd = torch.from_numpy(h).to(dev)
    sig = torch.empty((n, 65), dtype=torch.uint8, device=dev)
    exp = torch.empty((n, 20), dtype=torch.uint8, device=dev)
    assert lib.eges_synth_sign_msg_dev(0, 0, n, hd.data_ptr(), sig.data_ptr(), exp.data_ptr(), None) == 0
    torch.cuda.synchronize()
    from eges_amd.engine import pack_raw
    raw, off = pack_raw(txs.c1_raw(0, sig.cpu().numpy()))
    addr = np.zeros((n, 20), np.uint8)
    st = np.zeros(n, np.uint8)
    dev_in = os.environ.get("PHASES_WIRE_DEV") == "1"  # the bytes in device memory (the *_dev entry)
    if dev_in:
        rd = torch.from_numpy(raw).to(dev)
        od = torch.from_numpy(off.astype(np.int64)).to(dev)
        ad = torch.empty((n, 20), dtype=torch.uint8, device=dev)
        sd = torch.empty(n, dtype=torch.uint8, device=dev)
    for it in range(3):
        t0 = time.perf_counter()
        if dev_in:
            assert lib.eges_sender_raw_batch_dev(0, rd.data_ptr(), od.data_ptr(), n, 2, txs.GEEC_CHAIN_ID, ad.data_ptr(),
                                                 sd.data_ptr(), None, None) == 0, lib.eges_last_error()
            torch.cuda.synchronize()
        else:
            assert lib.eges_sender_raw_batch(raw.ctypes.data, off.ctypes.data, n, 2, txs.GEEC_CHAIN_ID, addr.ctypes.data,
                                             st.ctypes.data, None) == 0, lib.eges_last_error()
        dt = time.perf_counter() - t0
    if dev_in:
        addr[:] = ad.cpu().numpy()
        st[:] = sd.cpu().numpy()
    assert (addr == exp.cpu().numpy()).all() and int(st.max()) == 0, "diag build disagrees with the signer"
    return dt


def run_dev(n):
    msg = torch.empty(n * 32, dtype=torch.uint8, device=dev)
    sig = torch.empty(n * 65, dtype=torch.uint8, device=dev)
    exp = torch.empty(n * 20, dtype=torch.uint8, device=dev)
    addr = torch.empty(n * 20, dtype=torch.uint8, device=dev)
    status = torch.empty(n, dtype=torch.uint8, device=dev)
    assert lib.eges_synth_sign_dev(0, 0, n, msg.data_ptr(), sig.data_ptr(), exp.data_ptr(), None) == 0
    torch.cuda.synchronize()
    for it in range(3):
        t0 = time.perf_counter()
        assert lib.eges_ecrecover_batch_dev(0, msg.data_ptr(), sig.data_ptr(), n, None, addr.data_ptr(),
                                            status.data_ptr(), None) == 0, lib.eges_last_error()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
    assert bool((addr == exp).all()) and int(status.max()) == 0, "diag build disagrees with synth addresses"
    return dt


for n in [int(x) for x in (sys.argv[1:] or ["10000"])]:
    dt = run_wire(n) if WIRE else run_dev(n)
    rows = lib.eges_diag_read_stamps(None, 1 << 30)
    buf = (ctypes.c_uint64 * (rows * 8))()
    lib.eges_diag_read_stamps(buf, rows)
    a = np.frombuffer(buf, dtype=np.uint64).reshape(rows // 4, 4, 8).astype(np.float64)
    print(f"n={n} launch {dt * 1e3:.3f} ms (stamped build, host-timed), workgroups={rows // 4}, "
          f"form {'bucket' if FORM else 'windowed'}{', wire-format batch' if WIRE else ''}")
    for w, (name, ph) in ROLES.items():
        tot = a[:, w, :].sum(axis=1)
        print(f"  wave {w} ({name}): total mean {tot.mean():.4g} max {tot.max():.4g} ticks")
        for i, label in ph.items():
            print(f"      {label:22s} {a[:, w, i].mean():10.4g}  {100 * a[:, w, i].mean() / tot.mean():5.1f}%")
