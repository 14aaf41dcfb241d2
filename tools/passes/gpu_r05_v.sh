# Round-5 pass v: the default bench line twice on one box (the driver's N = 1 command), with the
# PMC file of the current sources in place (roofline.traffic), to set the evidence box's C2 beside another.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r05_v
mkdir -p $O
for i in 1 2; do
  timeout -k 10 300 python bench.py > $O/bench_$i.json 2> $O/bench_$i.err
  python - $O/bench_$i.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
r = d["roofline"]
print(d["value"], d["ms_per_step"], r["kernel_ms"], r["frac"], r.get("traffic"), d["secondary"]["c4_strong"]["sigs_per_s"], d["secondary"]["single"]["p50_ms_one_caller"], d["secondary"]["c3_block"]["median_ms"])
PY
done
echo done rc=0
