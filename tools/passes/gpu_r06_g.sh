# Round-6 pass g: the publication fixes on the product library: the tests of every path that
# publishes through a word (gate, resident, handoff, mid), then same-box A/Bs: C1 with the
# completion word + read-back (EGES_GATE_WORD=1) / the stream's completion signal (0) / round 5's
# word without read-back (tools/abprev); single recover p50 with output tags / without (abprev).
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r06_g
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_gate.py tests/test_gpu_resident.py tests/test_gpu_handoff.py tests/test_gpu_concurrency.py > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
for i in 1 2 3; do
  for v in w1 w0 prev; do
    L=; W=1
    [ $v = prev ] && L=tools/abprev/libeges.so
    [ $v = w0 ] && W=0
    EGES_AB_LIB=$L EGES_GATE_WORD=$W timeout -k 10 200 python bench.py --config c1 --steps 40 > $O/c1_${v}_$i.json 2> $O/c1_${v}_$i.err
    python -c "import json; a=json.load(open('$O/c1_${v}_$i.json')); print('c1 $v', a['value'], a['ms_per_batch'], a['p99_ms'], a['config']['correct'])"
  done
  for v in new prev; do
    S=tools/single_bench; [ $v = prev ] && S=tools/abprev/single_bench
    timeout -k 10 200 $S 1 3000 > $O/single_${v}_$i.json 2> $O/single_${v}_$i.err
    python -c "import json; a=json.load(open('$O/single_${v}_$i.json')); print('single $v', {k: a[k] for k in a if 'p50' in k or 'p99' in k})"
  done
done
timeout -k 10 200 tools/single_bench 16 2000 > $O/single16.json 2> $O/single16.err
cut -c1-400 $O/single16.json
echo done
