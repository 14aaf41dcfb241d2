# Wire-format path on the GPU: parity tests, then the C3 block latency from wire bytes. Run via gpurun.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_raw.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_raw.log 2>&1
timeout -k 10 200 python bench.py --config c3raw > gpurun_out/bench_c3raw.json 2> gpurun_out/bench_c3raw.err
timeout -k 10 200 python bench.py --config c3 > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err
tail -3 gpurun_out/pytest_raw.log
cat gpurun_out/bench_c3raw.json gpurun_out/bench_c3.json
