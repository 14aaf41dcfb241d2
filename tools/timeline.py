"""GPU timeline of host-buffer calls from a rocprofv3 --kernel-trace --memory-copy-trace run
(tools/passes/gpu_r05_i.sh): the recover_kernel launches and the copies between them, grouped into calls
(a gap of more than 1 ms between GPU operations starts a new call). Prints per call: its span from
the first copy to the last, the kernels' summed time, the idle time between kernels, and the copy
time not hidden behind a kernel (before the first and after the last)."""
import csv
import glob
import json
import os
import sys


def rows(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def col(r, *names):
    for n in names:
        if n in r:
            return r[n]
    raise KeyError(names)


def main(d):
    kt = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    mt = glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True)
    ev = []
    for r in rows(kt[0]):
        name = col(r, "Kernel_Name")
        if "eges::recover_kernel" not in name:
            continue
        ev.append(("K", int(col(r, "Start_Timestamp")), int(col(r, "End_Timestamp"))))
    for r in rows(mt[0]) if mt else []:
        dirn = col(r, "Direction", "Operation")
        ev.append(("H2D" if "HOST_TO_DEVICE" in dirn.upper() or "H2D" in dirn.upper() else "D2H",
                   int(col(r, "Start_Timestamp")), int(col(r, "End_Timestamp"))))
    ev.sort(key=lambda e: e[1])
    calls, cur = [], []
    for e in ev:
        if cur and e[1] - max(x[2] for x in cur) > 1_000_000:
            calls.append(cur)
            cur = []
        cur.append(e)
    if cur:
        calls.append(cur)
    out = []
    for c in calls:
        ks = [e for e in c if e[0] == "K"]
        if not ks:
            continue
        t0, t1 = min(e[1] for e in c), max(e[2] for e in c)
        busy = sum(e[2] - e[1] for e in ks)
        idle = sum(max(0, b[1] - a[2]) for a, b in zip(ks, ks[1:]))
        out.append({"kernels": len(ks), "span_ms": round((t1 - t0) / 1e6, 3), "kernel_ms": round(busy / 1e6, 3),
                    "between_kernels_ms": round(idle / 1e6, 3),
                    "before_first_kernel_ms": round((ks[0][1] - t0) / 1e6, 3),
                    "after_last_kernel_ms": round((t1 - ks[-1][2]) / 1e6, 3),
                    "copies": sum(1 for e in c if e[0] != "K"),
                    "copy_ms": round(sum(e[2] - e[1] for e in c if e[0] != "K") / 1e6, 3),
                    "kernel_each_ms": [round((e[2] - e[1]) / 1e6, 3) for e in ks]})
    for o in out:
        print(json.dumps(o))


if __name__ == "__main__":
    main(sys.argv[1])
