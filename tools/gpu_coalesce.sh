# Coalescer / latency check (via gpurun): concurrency + latency parity tests, the wave-0 and
# wave-1 phase breakdown of the latency kernel, and the native single-item bench with the
# gather window on and off (same box, alternating).
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_concurrency.py tests/test_gpu_lat.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_co.log 2>&1
tail -2 gpurun_out/pytest_co.log
timeout -k 10 120 python tools/phases.py 16 > gpurun_out/phases16.txt 2>&1
timeout -k 10 120 python tools/phases.py 1000 > gpurun_out/phases1000.txt 2>&1
cat gpurun_out/phases16.txt gpurun_out/phases1000.txt
for rep in 1 2; do
  for g in 0 20; do
    EGES_COALESCE_GATHER_US=$g timeout -k 10 120 tools/single_bench 8 2000 > gpurun_out/single_g${g}_$rep.json 2>> gpurun_out/single.err
    echo "gather=$g rep=$rep $(cat gpurun_out/single_g${g}_$rep.json)"
  done
done
timeout -k 10 120 tools/single_bench 16 2000 > gpurun_out/single16.json 2>> gpurun_out/single.err
cat gpurun_out/single16.json
