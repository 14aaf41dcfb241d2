# Latency-kernel check (via gpurun): latency / fr / concurrency / golden / block / raw parity
# tests, the stamped phase breakdown at n = 16 and 1000, the native single-item bench (8 and 16
# callers), the C3 block.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 180 python -u -m pytest tests/test_gpu_lat.py -m gpu -x -v --timeout 60 --timeout-method thread > gpurun_out/pytest_lat.log 2>&1 || { tail -30 gpurun_out/pytest_lat.log; exit 1; }
tail -1 gpurun_out/pytest_lat.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_fr.py tests/test_gpu_concurrency.py tests/test_gpu_parity.py tests/test_gpu_block.py tests/test_gpu_raw.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_more.log 2>&1 || { tail -30 gpurun_out/pytest_more.log; exit 1; }
tail -1 gpurun_out/pytest_more.log
timeout -k 10 120 python tools/phases.py 16 > gpurun_out/phases16.txt 2>&1
timeout -k 10 120 python tools/phases.py 1000 > gpurun_out/phases1000.txt 2>&1
tail -9 gpurun_out/phases16.txt; tail -9 gpurun_out/phases1000.txt
for rep in 1 2; do
  timeout -k 10 120 tools/single_bench 8 2000 > gpurun_out/single8_$rep.json 2>> gpurun_out/single.err
  cat gpurun_out/single8_$rep.json
done
timeout -k 10 120 tools/single_bench 16 2000 > gpurun_out/single16.json 2>> gpurun_out/single.err
timeout -k 10 200 python bench.py --config c3 --no-cpu-baseline > gpurun_out/c3.json 2> gpurun_out/c3.err
cat gpurun_out/single16.json gpurun_out/c3.json
