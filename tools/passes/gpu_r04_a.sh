# Round-4 first pass on one GPU (via gpurun): every GPU test, the latency microbenchmark, the
# default bench line. Outputs under gpurun_out/r04_a.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04_a
mkdir -p $O
timeout -k 10 120 tools/ubench_lat > $O/ubench_lat.txt 2>&1
cat $O/ubench_lat.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { tail -40 $O/pytest_gpu.txt; exit 1; }
tail -1 $O/pytest_gpu.txt
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
cat $O/bench.json
timeout -k 10 120 tools/block_bench 1000 300 > $O/block_bench.json 2>&1
cat $O/block_bench.json
timeout -k 10 120 tools/block_bench_diag 1000 300 > $O/block_bench_diag.json 2>&1
cat $O/block_bench_diag.json
