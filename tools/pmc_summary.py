"""Summarise tools/pmc.sh output into the schema bench.py reads (profiles/pmc_traffic.json): one
entry per (config, kernel) with that kernel's own launch size (`batch`: items per launch; the
counters' Grid_Size is kept beside it as a check), per-launch counter means, the L2 <-> fabric
traffic (FETCH_SIZE x 2 for the gfx950 16-byte-read correction + WRITE_SIZE, both KB -> bytes),
and the SHA-256 of the kernel sources the counters were collected from (bench.py refuses a
summary of other sources).

usage: python tools/pmc_summary.py <out.json> <config>:<kernel>:<batch>:<dir> [...]"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def summarise(root, kernel):
    """Per-dispatch counter sums of `kernel` in every pass under root, averaged over dispatches."""
    vals = defaultdict(list)
    grids = set()
    for f in glob.glob(f"{root}/pmc_*/run_counter_collection.csv") + glob.glob(f"{root}/pmc_*/*/run_counter_collection.csv"):
        per = defaultdict(float)
        for row in csv.DictReader(open(f)):
            if not row["Kernel_Name"].startswith(kernel + "("):
                continue
            per[(row["Dispatch_Id"], row["Counter_Name"])] += float(row["Counter_Value"])
            if row.get("Grid_Size"):
                grids.add(int(float(row["Grid_Size"])))
        for (d, c), v in per.items():
            vals[c].append(v)
    e = {c: sum(v) / len(v) for c, v in sorted(vals.items())}
    e["dispatches_per_counter"] = {c: len(v) for c, v in sorted(vals.items())}
    e["grid_sizes"] = sorted(grids)
    if "FETCH_SIZE" in e and "WRITE_SIZE" in e:
        e["fetch_bytes_x2"] = e["FETCH_SIZE"] * 1024 * 2
        e["write_bytes"] = e["WRITE_SIZE"] * 1024
        e["bytes_per_launch"] = round(e["fetch_bytes_x2"] + e["write_bytes"])
    return e


if __name__ == "__main__":
    from bench import kernel_src_hash
    out = sys.argv[1]
    entries = []
    for spec in sys.argv[2:]:
        cfg, rest = spec.split(":", 1)
        kernel, batch, root = rest.rsplit(":", 2)
        e = summarise(root, kernel)
        e.update(config=cfg, kernel=kernel, batch=int(batch))
        entries.append(e)
    doc = {"src_sha256": kernel_src_hash(), "git_head": os.environ.get("EGES_GIT_HEAD"),
           "collected_by": "tools/pmc.sh (one rocprofv3 --pmc pass per counter group, one bench.py config per "
                           "process, so each entry is one kernel at one launch size)",
           "note": "per launch: counters summed over the launch's XCDs, averaged over its dispatches; traffic = "
                   "FETCH_SIZE x 1024 x 2 (gfx950 correction) + WRITE_SIZE x 1024: bytes between L2 and the fabric "
                   "(Infinity Cache / HBM), not HBM alone",
           "entries": entries}
    js = json.dumps(doc, indent=1)
    open(out, "w").write(js + "\n")
    print(js)
