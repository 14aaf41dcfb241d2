# Round-5 pass z: the final tree (tools moved, PMC file for the current hash): every GPU test,
# smoke, and the default bench line (its roofline.traffic from profiles/pmc_traffic.json)
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r05_z
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
tail -1 $O/smoke.txt
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
python - $O/bench.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
r = d["roofline"]
print(d["value"], d["ms_per_step"], r["kernel_ms"], r["frac"], r.get("traffic"), d["secondary"]["c4_strong"]["sigs_per_s"],
      d["secondary"]["single"]["p50_ms_one_caller"], d["secondary"]["c3_block"]["median_ms"], d["secondary"]["c1_transfers"]["median_ms"])
PY
echo done rc=0
