#!/usr/bin/env python3
"""Host-buffer 1M ecrecover with the caller's arrays in pageable memory (numpy) against arrays in
pinned host memory (hipHostMalloc, here through torch's pin_memory allocator): HIP's copies from
pinned memory run on the copy engine directly (no staging, no blit kernels). Alternating, every
address checked. One JSON line per run."""
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
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    eges_amd.init(1)
    msg, sig, exp = eges_amd.synth_sign_dev(0, n, 0)
    torch.cuda.synchronize()
    page = {"msg": msg.cpu().numpy().copy(), "sig": sig.cpu().numpy().copy()}
    exp_h = exp.cpu().numpy()
    pin = {}
    for k, a in page.items():
        t = torch.empty(a.shape, dtype=torch.uint8, pin_memory=True)
        t.numpy()[:] = a
        pin[k] = t.numpy()
    outs = {"page": (np.zeros((n, 20), np.uint8), np.zeros(n, np.uint8)),
            "pin": (torch.empty((n, 20), dtype=torch.uint8, pin_memory=True).numpy(),
                    torch.empty(n, dtype=torch.uint8, pin_memory=True).numpy())}
    for rnd in range(3):
        for kind, src in (("page", page), ("pin", pin)):
            oa, os_ = outs[kind]
            for _ in range(2):
                eges_amd.ecrecover_batch(src["msg"], src["sig"], want_pub=False, out_addr=oa, out_status=os_)
            oa.fill(0)
            t0 = time.perf_counter()
            for _ in range(reps):
                _, addr, st = eges_amd.ecrecover_batch(src["msg"], src["sig"], want_pub=False, out_addr=oa, out_status=os_)
            dt = (time.perf_counter() - t0) / reps
            ok = bool((st == 0).all()) and np.array_equal(addr, exp_h)
            print(json.dumps({"round": rnd, "inputs": kind, "n": n, "ms_per_call": round(dt * 1e3, 3),
                              "sigs_per_s": round(n / dt, 1), "correct": ok}), flush=True)


if __name__ == "__main__":
    main()
