# Coalescer spinner cap A/B (EGES_COALESCE_SPINNERS) over 8..64 native caller threads.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_concurrency.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/pytest_co.log 2>&1
tail -1 gpurun_out/pytest_co.log
for t in ${THREADS:-8 16 32 64}; do
  for sp in ${CAPS:-1000 8}; do
    EGES_COALESCE_SPINNERS=$sp timeout -k 10 120 tools/single_bench $t 3000 > gpurun_out/sp_${t}_$sp.json 2>>gpurun_out/sp.err
    python -c "import json;b=json.load(open('gpurun_out/sp_${t}_$sp.json'));print('threads=$t spinners=$sp', b['recoveries_per_s'], b['errors'])"
  done
done
