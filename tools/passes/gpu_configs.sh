# All bench configs on one GPU (run via gpurun after tools/passes/gpu_check.sh).
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python bench.py --config c3 > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err
timeout -k 10 200 python bench.py --config c5 --steps 3 > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err
timeout -k 10 200 python bench.py --config verify --steps 3 > gpurun_out/bench_verify.json 2> gpurun_out/bench_verify.err
timeout -k 10 300 python bench.py --config c4 --steps 3 --warmup 1 > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err
cat gpurun_out/bench_c3.json gpurun_out/bench_c5.json gpurun_out/bench_verify.json gpurun_out/bench_c4.json
