# Round-5 pass i: every GPU test on the current sources (the resident idle-window test included),
# then the c2host call's GPU timeline: kernel + memory-copy trace of 8-chunk and 4-chunk calls.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r05_i
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
grep -E "other process 1M kernel" $O/pytest.txt || true
for pt in 8 4; do
  EGES_HOST_PARTS=$pt timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace -d $O/tl_$pt -o run --output-format csv -- python bench.py --config c2host --steps 4 --warmup 1 > $O/tl_$pt.log 2>&1
  find $O/tl_$pt -name "*.csv" | head
done
echo done rc=0
