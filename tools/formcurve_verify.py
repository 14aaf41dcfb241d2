#!/usr/bin/env python3
"""crypto.VerifySignature time by batch size for each verify form: the
product routing ("auto": latency kernels up to EGES_LAT_MAX, the bucket form's verify mode up to
64 x CUs, the lane-serial kernel above) against each form forced with engine knobs, one process.

  dev    device-resident eges_verify_batch_dev, HIP events on one stream, mean of REPS launches
  whole  host buffers through eges_verify_batch, median of REPS calls

Inputs: synthetic signatures, a quarter of the keys compressed; every call's 0/1 outputs are
checked against the expectation (all valid). Prints one JSON object per (n, form) and a summary."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

FORMS = {
    "auto": {},
    "auto_nob2": {"EGES_BKT2": 0},  # round 5's routing: no two-per-CU bucket form
    "auto2": {"EGES_VERIFY_MID_GENS": 2},  # the bucket form for up to two generations of workgroups
    "lat": {"EGES_LAT_MAX": 1 << 20},
    "bucket": {"EGES_LAT_MAX": 0, "EGES_MID_MAX": 1 << 20, "EGES_MID_FORM": 2},
    "b2": {"EGES_LAT_MAX": 0, "EGES_MID_MAX": 1 << 20, "EGES_MID_FORM": 2, "EGES_BKT2": 2},
    "lane": {"EGES_LAT_MAX": 0, "EGES_MID_MAX": 0},
}


def main():
    import torch

    import eges_amd
    sizes = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else
                              "1000,2000,4096,8192,12000,16384,24000,40000,65536,100000").split(",")]
    reps = int(os.environ.get("FORMCURVE_REPS", "10"))
    lat_cap = int(os.environ.get("FORMCURVE_LAT_CAP", "8192"))
    eges_amd.init(1)
    nmax = max(sizes)
    msg, sig, _ = eges_amd.synth_sign_dev(1 << 30, nmax, 0)
    pub = torch.empty((nmax, 65), dtype=torch.uint8, device="cuda")
    eges_amd.ecrecover_batch_dev(msg, sig, pub=pub)
    torch.cuda.synchronize()
    pub_h, sig_h, msg_h = pub.cpu().numpy(), sig.cpu().numpy()[:, :64].copy(), msg.cpu().numpy()
    publen = np.full(nmax, 65, np.uint8)
    comp = np.arange(nmax) % 4 == 3
    pub_h[comp, 0] = 2 + (pub_h[comp, 64] & 1)
    pub_h[comp, 33:] = 0
    publen[comp] = 33
    dp, dl, dm, ds = (torch.from_numpy(x).cuda() for x in (pub_h, publen, msg_h, sig_h))
    stream = torch.cuda.Stream()
    out = []
    for n in sizes:
        only = os.environ.get("FORMCURVE_FORMS")
        for form, kv in FORMS.items():
            if only and form not in only.split(","):
                continue
            if form == "lat" and n > lat_cap:
                continue
            old = {k: eges_amd.get_knob(k) for k in kv}
            for k, v in kv.items():
                eges_amd.set_knob(k, v)
            try:
                ok_d = torch.empty((n,), dtype=torch.uint8, device="cuda")
                evs = []
                for i in range(reps + 2):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(stream)
                    eges_amd.verify_batch_dev(dp[:n], dl[:n], dm[:n], ds[:n], ok=ok_d, stream=stream.cuda_stream)
                    e1.record(stream)
                    if i >= 2:
                        evs.append((e0, e1))
                torch.cuda.synchronize()
                dev_ms = sum(a.elapsed_time(b) for a, b in evs) / len(evs)
                ok = bool((ok_d == 1).all().item())
                lat = []
                for i in range(reps + 2):
                    t0 = time.perf_counter()
                    r = eges_amd.verify_batch(pub_h[:n], publen[:n], msg_h[:n], sig_h[:n])
                    dt = time.perf_counter() - t0
                    if i >= 2:
                        lat.append(dt)
                    ok = ok and bool((r == 1).all())
            finally:
                for k, v in old.items():
                    eges_amd.set_knob(k, v)
            rec = {"n": n, "form": form, "dev_ms": round(dev_ms, 4), "whole_ms": round(float(np.median(lat)) * 1e3, 4),
                   "dev_sigs_per_s": round(n / (dev_ms / 1e3), 1), "correct": ok}
            out.append(rec)
            print(json.dumps(rec), flush=True)
    print(json.dumps({"summary_auto_dev_ms": {str(r["n"]): r["dev_ms"] for r in out if r["form"] == "auto"},
                      "all_correct": all(r["correct"] for r in out)}), flush=True)


if __name__ == "__main__":
    main()
