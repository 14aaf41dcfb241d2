# C1 iteration: wire-path parity tests (both forms), C1 bench + kernel stats, bucket phases.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/c1w_${1:-a}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_raw.py tests/test_gpu_rlp.py tests/test_gpu_block.py tests/test_c1.py tests/test_gpu_mid.py -x -v --timeout 200 --timeout-method thread > $O/pytest_wire.log 2>&1 || { tail -60 $O/pytest_wire.log; exit 1; }
tail -2 $O/pytest_wire.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --config c1 --no-cpu-baseline --steps 20 > $O/c1.json 2> $O/c1.err
cat $O/c1.json
find $O/prof -name "*kernel_stats.csv" -exec head -3 {} \;
for i in 1 2; do timeout -k 10 200 python bench.py --config c1 --no-cpu-baseline > $O/c1_$i.json 2>> $O/c1.err; cat $O/c1_$i.json | python -c "import json,sys; d=json.load(sys.stdin); print('c1', d['ms_per_batch'], d['p99_ms'])"; done
timeout -k 10 200 python tools/phases_mid.py 10000 > $O/phases.txt 2>&1
cat $O/phases.txt
for v in ${2:-}; do
  EGES_DIAG_LIB=libeges_diag_$v.so timeout -k 10 200 python tools/phases_mid.py 10000 > $O/phases_$v.txt 2>&1
  echo "== variant $v"; cat $O/phases_$v.txt
done
