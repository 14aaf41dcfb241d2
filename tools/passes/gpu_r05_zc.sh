# Round-5 pass zc: the windowed form capped at one generation in auto routing. Every GPU test,
# smoke, the routing curve around the cut, the PMC passes for the new source hash, the bench line.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r05_zc
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
tail -1 $O/smoke.txt
FORMCURVE_FORMS=auto FORMCURVE_REPS=12 timeout -k 10 300 python -u tools/formcurve.py 24000,32768,33000,36000,40000 > $O/formcurve_auto_cut.jsonl
cat $O/formcurve_auto_cut.jsonl
bash tools/pmc.sh > $O/pmc.log 2>&1
tail -1 $O/pmc.log
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
python - $O/bench.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
r = d["roofline"]
print(d["value"], r["kernel_ms"], r["frac"], r.get("traffic"), d["secondary"]["c3_block"]["median_ms"], d["secondary"]["c1_transfers"]["median_ms"])
PY
echo done rc=0
