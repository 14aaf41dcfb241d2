# Round-5 pass l: every GPU test on the current sources (progressive gate on, resident idle window 1 ms,
# the two-process idle-window test), smoke, and the single-call seam at the new window.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r05_l
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -s > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
grep -E "other process 1M kernel" $O/pytest.txt || true
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
tail -1 $O/smoke.txt
timeout -k 10 120 tools/single_bench 16 2000 > $O/single16.json 2>/dev/null
tail -1 $O/single16.json
echo done rc=0
