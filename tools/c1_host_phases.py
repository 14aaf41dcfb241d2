#!/usr/bin/env python3
"""C1 (10k wire-format transfers through eges_sender_raw_batch) timed around the C-ABI call, with
the engine's host phase split (hostpath.hip HSTAMP: acquire, pack, launch, sync, unpack) from the
stamped diagnostic build. Run with EGES_AB_LIB=eges_amd/libeges_diag.so (the stamped kernels are
slower; the host phases are what this reads). Prints one JSON line.
usage: EGES_AB_LIB=$PWD/eges_amd/libeges_diag.so python tools/c1_host_phases.py [n=10000] [iters=100]"""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import eges_amd
    from eges_amd import txs
    from eges_amd._lib import SIGNER_EIP155, check, lib
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 100
    eges_amd.init(1)
    h = txs.c1_sighashes(0, n)
    sig_d, exp_d = eges_amd.synth_sign_msg_dev(torch.from_numpy(h).cuda(), 0)
    torch.cuda.synchronize()
    sig_h, exp_h = sig_d.cpu().numpy(), exp_d.cpu().numpy()
    raw, offs = eges_amd.pack_raw(txs.c1_raw(0, sig_h))
    P = lambda a: ctypes.c_void_p(a.ctypes.data)  # noqa: E731
    addr = np.zeros((n, 20), np.uint8)
    st = np.zeros(n, np.uint8)
    stamps = getattr(lib, "eges_diag_host_stamps", None)
    if stamps is not None:
        stamps.restype = ctypes.c_size_t
    t = (ctypes.c_int64 * 6)()
    lat, ph = [], []
    ok = True
    for i in range(iters + 10):
        t0 = time.perf_counter()
        rc = lib.eges_sender_raw_batch(P(raw), P(offs), n, SIGNER_EIP155, txs.GEEC_CHAIN_ID, P(addr), P(st), None)
        dt = time.perf_counter() - t0
        check(rc)
        ok = ok and bool((st == 0).all()) and np.array_equal(addr, exp_h)
        if i < 10:
            continue
        lat.append(dt * 1e3)
        if stamps is not None:
            stamps(t, 6)
            ph.append([(t[k + 1] - t[k]) / 1e3 for k in range(5)])
    out = {"metric": "C1 via eges_sender_raw_batch, ctypes caller", "txs": n, "iters": iters,
           "median_ms": round(float(np.median(lat)), 4), "correct": ok}
    if ph:
        a = np.median(np.array(ph), axis=0)
        out["host_phases_us_median"] = dict(zip(["acquire", "pack", "launch", "sync", "unpack"],
                                                [round(float(x), 2) for x in a]))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
