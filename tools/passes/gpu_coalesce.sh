# Coalescer check (via gpurun): concurrency tests, then the native single-item bench at 8 and 16
# callers with the gather window on and off (same box, alternating).
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_concurrency.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_co.log 2>&1
tail -1 gpurun_out/pytest_co.log
for rep in 1 2; do
  for g in 0 20; do
    EGES_COALESCE_GATHER_US=$g timeout -k 10 120 tools/single_bench 8 2000 > gpurun_out/single_g${g}_$rep.json 2>> gpurun_out/single.err
    echo "gather=$g rep=$rep $(cat gpurun_out/single_g${g}_$rep.json)"
  done
done
timeout -k 10 120 tools/single_bench 16 2000 > gpurun_out/single16.json 2>> gpurun_out/single.err
cat gpurun_out/single16.json
