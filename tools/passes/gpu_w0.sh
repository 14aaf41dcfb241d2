# Split point sweep (via gpurun): latency tests on the default build, then the stamped n = 16
# per-wave totals of diagnostic builds with EGES_SPLIT_W0 = 14 / 15 (default) / 16, alternating.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 180 python -u -m pytest tests/test_gpu_lat.py tests/test_gpu_concurrency.py -m gpu -x -q --timeout 100 --timeout-method thread > gpurun_out/pytest_lat.log 2>&1 || { tail -30 gpurun_out/pytest_lat.log; exit 1; }
tail -1 gpurun_out/pytest_lat.log
for rep in 1 2; do
  for lib in libeges_diag_w14.so libeges_diag.so libeges_diag_w16.so; do
    EGES_DIAG_LIB=$lib timeout -k 10 100 python tools/phases.py 16 > gpurun_out/w0_$lib.txt 2>&1
    echo "$lib $(grep -E 'per-wave' gpurun_out/w0_$lib.txt)"
  done
done
tail -9 gpurun_out/w0_libeges_diag.so.txt
timeout -k 10 120 tools/single_bench 8 2000 > gpurun_out/single8.json 2>> gpurun_out/single.err
timeout -k 10 120 tools/single_bench 16 2000 > gpurun_out/single16.json 2>> gpurun_out/single.err
cat gpurun_out/single8.json gpurun_out/single16.json
