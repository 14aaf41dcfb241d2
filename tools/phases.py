"""Phase breakdown of the recover kernel (diagnostic build eges_amd/libeges_diag.so).

Runs one 1M-signature ecrecover launch through the phase-stamped kernel and prints, per
phase, the mean s_memtime cycles each wave spent there and the share of the total.
Usage: python tools/phases.py [n]
"""
import ctypes
import os
import sys
import time

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

LAT = False
PHASES = ["parse+sqrt", "r^-1 batch+u1/u2", "GLV+digits", "R table+affine", "Strauss", "Z^-1 batch",
          "keccak+store", "-"]

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
if n <= int(os.environ.get("EGES_LAT_MAX", "8192")):  # the latency kernel's phases (k_recover_lat.hip)
    PHASES = ["parse + x, c", "wait: wave 1 r^-1+digits", "(wave 1: r^-1)", "R' table", "Strauss + join",
              "Z^-1+affine", "keccak+store", "(wave 1: u1,u2,GLV,digits)"]
    LAT = True
assert lib.eges_init(0, 0) == 0, lib.eges_last_error()
dev = torch.device("cuda:0")
msg = torch.empty(n * 32, dtype=torch.uint8, device=dev)
sig = torch.empty(n * 65, dtype=torch.uint8, device=dev)
exp = torch.empty(n * 20, dtype=torch.uint8, device=dev)
addr = torch.empty(n * 20, dtype=torch.uint8, device=dev)
status = torch.empty(n, dtype=torch.uint8, device=dev)
torch.cuda.synchronize()
assert lib.eges_synth_sign_dev(0, 0, n, msg.data_ptr(), sig.data_ptr(), exp.data_ptr(), None) == 0
torch.cuda.synchronize()
for it in range(2):
    t0 = time.perf_counter()
    rc = lib.eges_ecrecover_batch_dev(0, msg.data_ptr(), sig.data_ptr(), n, None, addr.data_ptr(),
                                      status.data_ptr(), None)
    assert rc == 0, lib.eges_last_error()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
if not os.environ.get("EGES_PROBE"):  # probe builds compute wrong results on purpose
    assert bool((addr == exp).all()) and int(status.max()) == 0, "diag build disagrees with synth addresses"
waves = lib.eges_diag_read_stamps(None, 1 << 30)
buf = (ctypes.c_uint64 * (waves * 8))()
lib.eges_diag_read_stamps(buf, waves)
import numpy as np  # noqa: E402

raw = np.frombuffer(buf, dtype=np.uint64).reshape(waves, 8)
place = None
if LAT:  # slots 2 / 7 carry wave 1's / wave 0's hw_place in their high words (k_recover_lat.hip)
    place = (raw[:, [2, 7]] >> np.uint64(32)).astype(np.int64)
    raw = raw.copy()
    raw[:, [2, 7]] &= np.uint64(0xFFFFFFFF)
a = raw.astype(np.float64)
tot = (a.sum(axis=1) - a[:, 2] - a[:, 7]) if LAT else a.sum(axis=1)
print(f"n={n} launch {dt * 1e3:.2f} ms ({n / dt / 1e6:.2f} M sigs/s, stamped build), waves={waves}")
print(f"per-wave total: mean {tot.mean():.4g} min {tot.min():.4g} max {tot.max():.4g} (s_memtime ticks)")
tiles_per_wave = max(n / 256 / (waves / 4), 1e-9)
for i in range(8 if LAT else 7):
    m = a[:, i].mean()
    print(f"  {PHASES[i]:18s} {m:12.4g} ticks/wave  {100 * m / tot.mean():5.1f}%  {m / tiles_per_wave:10.4g}/tile")

if place is not None and place.any():
    # SIMD sharing: key = (XCC, SE, SH, CU, SIMD); wave 0 is the heavy chain, wave 1 the scalar one
    def key(h):
        return (h >> 16, (h >> 13) & 7, (h >> 12) & 1, (h >> 8) & 15, (h >> 4) & 3)
    from collections import Counter
    heavy = Counter(key(int(h)) for h in place[:, 1])
    light = Counter(key(int(h)) for h in place[:, 0])
    cus = Counter(key(int(h))[:4] for h in place[:, 1])
    print(f"placement: {len(cus)} CUs, {len(heavy)} SIMDs with a wave 0; signatures per CU "
          f"{sorted(Counter(cus.values()).items())}; same-SIMD wave 0 / wave 1 pairs "
          f"{sum(key(int(p0)) == key(int(p1)) for p1, p0 in place)}")
    groups = {}
    for i, (p1, p0) in enumerate(place):
        k = key(int(p0))
        groups.setdefault((heavy[k], light.get(k, 0)), []).append(i)
    for (h, l), ix in sorted(groups.items()):
        print(f"  SIMD with {h} wave-0s and {l} wave-1s: {len(ix):5d} signatures, Strauss {a[ix, 4].mean():.4g}, "
              f"total {tot[ix].mean():.4g} ticks")
    sims = Counter(int(h) >> 4 & 3 for h in place[:, 1])
    print(f"  wave 0 SIMD ids {sorted(sims.items())}; wave 1 SIMD ids "
          f"{sorted(Counter(int(h) >> 4 & 3 for h in place[:, 0]).items())}")
