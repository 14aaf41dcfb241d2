#!/usr/bin/env python3
"""Whole-call and kernel time by batch size for each recover form (latency / mid-size /
lane-serial), selected with engine knobs in one process (tools/passes/gpu_formcurve.sh).

  whole  C1-shaped wire-format transfers through eges_sender_raw_batch (pageable host buffers:
         H2D + decode + sighash + recovery + D2H), median of REPS calls
  dev    device-resident eges_ecrecover_batch_dev (prep if any + recover), HIP events on the
         engine's stream, mean of REPS launches

Prints one JSON object per (n, form) and a summary line; every call's statuses / addresses are
checked against the synthetic signer's."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

FORMS = {
    "auto": {},  # the product routing (latency / mid-size / lane-serial by batch size)
    "auto_nob2": {"EGES_BKT2": 0},  # round 5's routing: no two-per-CU bucket form
    "b2": {"EGES_LAT_MAX": 0, "EGES_MID_MAX": 1 << 20, "EGES_MID_FORM": 2, "EGES_BKT2": 2},
    "lat": {"EGES_LAT_MAX": 1 << 20, "EGES_MID_MAX": 0},
    "mid": {"EGES_LAT_MAX": 0, "EGES_MID_MAX": 1 << 20, "EGES_MID_FORM": 2},
    "midw": {"EGES_LAT_MAX": 0, "EGES_MID_MAX": 1 << 20, "EGES_MID_FORM": 0},
    "midnf": {"EGES_LAT_MAX": 0, "EGES_MID_MAX": 1 << 20, "EGES_MID_FORM": 2, "EGES_WIRE_FUSED": 0},
    "lane": {"EGES_LAT_MAX": 0, "EGES_MID_MAX": 0},
}


def main():
    import torch

    import eges_amd
    from eges_amd import txs
    from eges_amd._lib import SIGNER_EIP155
    sizes = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else
                              "1000,2000,3000,4096,6000,8192,10000,16384,24000,32768,50000,65536,100000,131072").split(",")]
    lat_cap = int(os.environ.get("FORMCURVE_LAT_CAP", "16384"))
    reps = int(os.environ.get("FORMCURVE_REPS", "15"))
    eges_amd.init(1)
    nmax = max(sizes)
    sighash = txs.c1_sighashes(0, nmax)
    sig_d, exp_d = eges_amd.synth_sign_msg_dev(torch.from_numpy(sighash).cuda(), 0)
    torch.cuda.synchronize()
    sig_h, exp_h = sig_d.cpu().numpy(), exp_d.cpu().numpy()
    msg_d = torch.from_numpy(sighash).cuda()
    stream = torch.cuda.Stream()
    raws = txs.c1_raw(0, sig_h)
    out = []
    for n in sizes:
        packed = eges_amd.pack_raw(raws[:n])
        for form, kv in FORMS.items():
            if form not in os.environ.get("FORMCURVE_FORMS", "lat,mid,midw,lane").split(","):
                continue
            if form == "lat" and n > lat_cap:
                continue
            old = {k: eges_amd.get_knob(k) for k in kv}
            for k, v in kv.items():
                eges_amd.set_knob(k, v)
            try:
                ok = True
                lat = []
                for i in range(reps + 2):
                    t0 = time.perf_counter()
                    addr, st, _ = eges_amd.sender_raw_batch(packed, SIGNER_EIP155, txs.GEEC_CHAIN_ID)
                    dt = time.perf_counter() - t0
                    if i >= 2:
                        lat.append(dt)
                    ok = ok and bool((st == 0).all()) and np.array_equal(addr, exp_h[:n])
                addr_d = torch.empty((n, 20), dtype=torch.uint8, device="cuda")
                st_d = torch.empty((n,), dtype=torch.uint8, device="cuda")
                evs = []
                for i in range(reps + 2):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(stream)
                    eges_amd.ecrecover_batch_dev(msg_d[:n], sig_d[:n], addr=addr_d, status=st_d, stream=stream.cuda_stream)
                    e1.record(stream)
                    if i >= 2:
                        evs.append((e0, e1))
                torch.cuda.synchronize()
                dev_ms = sum(a.elapsed_time(b) for a, b in evs) / len(evs)
                ok = ok and bool((st_d == 0).all().item()) and bool(torch.equal(addr_d, exp_d[:n]))
            finally:
                for k, v in old.items():
                    eges_amd.set_knob(k, v)
            rec = {"n": n, "form": form, "whole_ms": round(float(np.median(lat)) * 1e3, 4),
                   "whole_p90_ms": round(float(np.percentile(lat, 90)) * 1e3, 4), "dev_ms": round(dev_ms, 4),
                   "whole_txs_per_s": round(n / float(np.median(lat)), 1), "correct": ok}
            out.append(rec)
            print(json.dumps(rec), flush=True)
    best = {}
    for r in out:
        b = best.get(r["n"])
        if b is None or r["whole_ms"] < b["whole_ms"]:
            best[r["n"]] = r
    print(json.dumps({"summary": {str(n): [b["form"], b["whole_ms"]] for n, b in sorted(best.items())},
                      "all_correct": all(r["correct"] for r in out)}), flush=True)


if __name__ == "__main__":
    main()
