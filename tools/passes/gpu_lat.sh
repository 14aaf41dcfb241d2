# Latency-kernel check (via gpurun): fr / latency / block / golden parity tests, the stamped
# phase breakdown at n = 1000 and 16, the C3 block bench and the native single-item bench.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_fr.py tests/test_gpu_lat.py tests/test_gpu_block.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_lat.log 2>&1
tail -2 gpurun_out/pytest_lat.log
timeout -k 10 120 python tools/phases.py 1000 > gpurun_out/phases_lat.txt 2>&1
timeout -k 10 120 python tools/phases.py 16 > gpurun_out/phases_lat16.txt 2>&1
timeout -k 10 200 python bench.py --config c3 > gpurun_out/c3.json 2> gpurun_out/c3.err
timeout -k 10 200 tools/single_bench 8 2000 > gpurun_out/single.json 2> gpurun_out/single.err
cat gpurun_out/c3.json gpurun_out/single.json
grep -A8 "per-wave" gpurun_out/phases_lat.txt
