"""Probe of the one-launch host-buffer form (hostpath.hip run_host_one) on the GPU box: 1M-signature
calls alternating two different synthetic batches, under every EGES_TEST_HOST_ONE mode (bit 0:
re-read the pinned outputs after the stream drained and fail the call if a copied block changed;
bit 1: coherent output memory; bit 2: non-temporal staging stores). Prints, per mode, the calls,
the wrongly returned items and the recheck failures: which side (the inputs the kernel read, or
the outputs this thread copied) a stale byte came from."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import eges_amd
    from eges_amd._lib import EgesError
    eges_amd.init(1)
    eges_amd.set_knob("EGES_HOST_ONE", 1)
    n = 1 << 20
    sets = []
    for first in (123_456_789, 987_654_321):
        msg, sig, exp = eges_amd.synth_sign_dev(first, n, 0)
        torch.cuda.synchronize()
        sets.append((msg.cpu().numpy(), sig.cpu().numpy(), exp.cpu().numpy()))
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    modes = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [1, 3, 5, 7]
    oa, os_ = np.zeros((n, 20), np.uint8), np.zeros(n, np.uint8)
    for mode in modes:
        eges_amd.set_knob("EGES_TEST_HOST_ONE", mode)
        wrong, rech, errs, first = 0, 0, [], []
        for i in range(reps):
            mh, sh, eh = sets[i % 2]
            os_.fill(0xEE)
            try:
                eges_amd.ecrecover_batch(mh, sh, want_pub=False, out_addr=oa, out_status=os_)
            except EgesError as e:
                rech += 1
                errs.append(str(e)[:120])
            bad = np.nonzero((oa != eh).any(axis=1) | (os_ != 0))[0]
            wrong += int(bad.size)
            if bad.size:
                first.append(bad[:4].tolist())
        t0 = time.perf_counter()
        for i in range(4):
            mh, sh, eh = sets[i % 2]
            try:
                eges_amd.ecrecover_batch(mh, sh, want_pub=False, out_addr=oa, out_status=os_)
            except EgesError:
                pass
        ms = (time.perf_counter() - t0) / 4 * 1e3
        print(json.dumps({"mode": mode, "calls": reps, "wrong_items": wrong, "recheck_failures": rech, "ms_per_call": round(ms, 3),
                          "errors": errs[:3], "first_bad": first[:4]}), flush=True)
    eges_amd.set_knob("EGES_TEST_HOST_ONE", 0)


if __name__ == "__main__":
    main()
