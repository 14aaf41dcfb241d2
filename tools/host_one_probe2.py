"""Round-6 probe of round 5's one-launch host form (profiles/r05/removed_host_one_r05.diff, rebuilt
from commit f000a43 with three discriminating test bits into tools/abhostone/libeges.so, loaded
through EGES_AB_LIB; never the product library). 1M-signature calls alternating two synthetic
batches; per EGES_TEST_HOST_ONE mode: calls, wrongly returned items, how many of them hold the
OTHER batch's address (the previous call's bytes) or zeros, the recheck's split into items a
second read right after the copy already had right vs still stale (bit 5), with bit 4 (20 us
between a block's done word and its copy) and bit 6 (each thread reads its items' last address
dword back at system scope before the block's done word)."""
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
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    modes = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [1, 33, 17, 65, 97]
    oa, os_ = np.zeros((n, 20), np.uint8), np.zeros(n, np.uint8)
    for mode in modes:
        eges_amd.set_knob("EGES_TEST_HOST_ONE", mode)
        wrong = prev = zeros = rech = 0
        errs, first, blocks = [], [], []
        t0 = time.perf_counter()
        for i in range(reps):
            mh, sh, eh = sets[i % 2]
            other = sets[(i + 1) % 2][2]
            os_.fill(0xEE)
            try:
                eges_amd.ecrecover_batch(mh, sh, want_pub=False, out_addr=oa, out_status=os_)
            except EgesError as e:
                rech += 1
                errs.append(str(e)[:200])
            bad = np.nonzero((oa != eh).any(axis=1) | (os_ != 0))[0]
            wrong += int(bad.size)
            if bad.size:
                prev += int((oa[bad] == other[bad]).all(axis=1).sum())
                zeros += int((oa[bad] == 0).all(axis=1).sum())
                first.append(bad[:3].tolist())
                gt = 262144
                blocks.extend(sorted({(int(b) // gt, (int(b) % gt) // 256) for b in bad})[:4])
        ms = (time.perf_counter() - t0) / reps * 1e3
        print(json.dumps({"mode": mode, "calls": reps, "wrong_items": wrong, "previous_call_bytes": prev, "zeros": zeros,
                          "recheck_failures": rech, "ms_per_call": round(ms, 3), "errors": errs[:4], "first_bad": first[:4],
                          "slot_block": blocks[:12]}), flush=True)
    eges_amd.set_knob("EGES_TEST_HOST_ONE", 0)


if __name__ == "__main__":
    main()
