# Full GPU pass (via gpurun): every -m gpu test, then the latency numbers (C3 block, single-item).
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 200 python bench.py --config c3 > gpurun_out/c3.json 2> gpurun_out/c3.err
timeout -k 10 200 tools/single_bench 8 2000 > gpurun_out/single.json 2> gpurun_out/single.err
timeout -k 10 200 tools/single_bench 16 2000 > gpurun_out/single16.json 2> gpurun_out/single16.err
cat gpurun_out/c3.json gpurun_out/single.json gpurun_out/single16.json
