"""Summarise tools/pmc.sh output: per-launch counter means for one kernel -> JSON on stdout."""
import csv
import glob
import json
import sys
from collections import defaultdict

kern = sys.argv[1] if len(sys.argv) > 1 else "eges::recover_kernel"
root = sys.argv[2] if len(sys.argv) > 2 else "gpurun_out"
vals = defaultdict(list)
for f in glob.glob(f"{root}/pmc_*/run_counter_collection.csv"):
    per = defaultdict(float)
    for row in csv.DictReader(open(f)):
        if not row["Kernel_Name"].startswith(kern):
            continue
        per[(row["Dispatch_Id"], row["Counter_Name"])] += float(row["Counter_Value"])
    for (d, c), v in per.items():
        vals[c].append(v)
out = {c: sum(v) / len(v) for c, v in sorted(vals.items())}
print(json.dumps(out, indent=1))
