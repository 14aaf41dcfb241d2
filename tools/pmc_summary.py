"""Summarise tools/pmc.sh output into the schema bench.py reads (profiles/pmc_traffic.json):
per-launch counter means for each kernel, the HBM-side traffic (FETCH_SIZE x 2 for the gfx950
16-byte-read correction + WRITE_SIZE, both KB -> bytes), and the SHA-256 of the kernel sources
the counters were collected from (bench.py refuses a summary of other sources).

usage: python tools/pmc_summary.py <gpurun_out dir> <batch> [out.json]"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
KERNELS = ("eges::recover_kernel", "eges::verify_kernel", "eges::recover_lat_kernel", "eges::recover_bkt_kernel",
           "eges::recover_mid_kernel")


def summarise(root):
    vals = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(f"{root}/pmc_*/run_counter_collection.csv"):
        per = defaultdict(float)
        names = {}
        for row in csv.DictReader(open(f)):
            k = next((k for k in KERNELS if row["Kernel_Name"].startswith(k)), None)
            if k is None:
                continue
            per[(k, row["Dispatch_Id"], row["Counter_Name"])] += float(row["Counter_Value"])
            names[k] = True
        for (k, d, c), v in per.items():
            vals[k][c].append(v)
    out = {}
    for k, cs in vals.items():
        e = {c: sum(v) / len(v) for c, v in sorted(cs.items())}
        if "FETCH_SIZE" in e and "WRITE_SIZE" in e:
            e["fetch_bytes_x2"] = e["FETCH_SIZE"] * 1024 * 2
            e["write_bytes"] = e["WRITE_SIZE"] * 1024
            e["bytes_per_launch"] = round(e["fetch_bytes_x2"] + e["write_bytes"])
        out[k] = e
    return out


if __name__ == "__main__":
    from bench import kernel_src_hash
    root, batch = sys.argv[1], int(sys.argv[2])
    ks = summarise(root)
    for e in ks.values():
        e["batch"] = batch
    doc = {"src_sha256": kernel_src_hash(), "git_head": os.environ.get("EGES_GIT_HEAD"),
           "collected_by": "tools/pmc.sh (one rocprofv3 --pmc pass per counter group over bench.py)",
           "note": "traffic = FETCH_SIZE x 1024 x 2 (gfx950 correction) + WRITE_SIZE x 1024 per launch: bytes "
                   "between L2 and the fabric (Infinity Cache / HBM), not HBM alone",
           "kernels": ks}
    js = json.dumps(doc, indent=1)
    if len(sys.argv) > 3:
        open(sys.argv[3], "w").write(js + "\n")
    print(js)
