#!/usr/bin/env python3
"""Where a small synchronous call's time goes outside its kernel, from one
`rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv` run of tools/block_bench:

  launch_api   the launching HIP call's own duration (host)
  to_start     launching call's start -> the kernel's start (host launch + CP dispatch)
  kernel       the kernel's duration
  to_return    the kernel's end -> the end of the next host synchronisation call on that thread
  call         launching call's start -> that synchronisation's end

usage: launch_gaps.py <dir with *_kernel_trace.csv and *_hip_api_trace.csv> [kernel substring]"""
import csv
import glob
import json
import os
import sys

import numpy as np


def main():
    d = sys.argv[1]
    want = sys.argv[2] if len(sys.argv) > 2 else "recover_lat_kernel"
    kt = list(csv.DictReader(open(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0])))
    at = list(csv.DictReader(open(glob.glob(os.path.join(d, "**", "*hip_api_trace.csv"), recursive=True)[0])))
    by_corr = {r["Correlation_Id"]: r for r in at}
    syncs = {}
    for r in at:
        if "Synchronize" in r["Function"]:
            syncs.setdefault(r["Thread_Id"], []).append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    for v in syncs.values():
        v.sort()
    rows = []
    for k in kt:
        if want not in k["Kernel_Name"]:
            continue
        api = by_corr.get(k["Correlation_Id"])
        if api is None:
            continue
        ks, ke = int(k["Start_Timestamp"]), int(k["End_Timestamp"])
        a0, a1 = int(api["Start_Timestamp"]), int(api["End_Timestamp"])
        nxt = [s for s in syncs.get(api["Thread_Id"], []) if s[1] >= ke]
        if not nxt:
            continue
        se = nxt[0][1]
        rows.append((a1 - a0, ks - a0, ke - ks, se - ke, se - a0))
    a = np.array(rows, dtype=np.float64) / 1e3  # us
    names = ["launch_api", "to_start", "kernel", "to_return", "call"]
    out = {"kernel": want, "calls": len(rows),
           "median_us": {n: round(float(np.median(a[:, i])), 2) for i, n in enumerate(names)},
           "p90_us": {n: round(float(np.percentile(a[:, i], 90)), 2) for i, n in enumerate(names)}}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
