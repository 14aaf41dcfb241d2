# Round-6 closing pass on the final sources: every GPU test, smoke, the PMC passes (tools/pmc.sh:
# profiles/pmc_traffic.json must match these kernel sources) and the default bench line.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/ev6_final3
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
bash tools/pmc.sh > $O/pmc.log 2>&1
cp gpurun_out/pmc_traffic.json $O/
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
head -c 300 $O/bench.json
