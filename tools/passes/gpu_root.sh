# Root-helper check (via gpurun): latency / parity / block / raw / concurrency tests, the narrow
# (eges_amd/libeges_diag_prev.so: the diagnostic build of the previous commit, built by hand)
# form's launch time at n = 1000 / 4096 / 8192 against the previous build (alternating), C3.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 180 python -u -m pytest tests/test_gpu_lat.py -m gpu -x -v --timeout 60 --timeout-method thread > gpurun_out/pytest_lat.log 2>&1 || { tail -30 gpurun_out/pytest_lat.log; exit 1; }
tail -1 gpurun_out/pytest_lat.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_block.py tests/test_gpu_raw.py tests/test_gpu_concurrency.py tests/test_gpu_rlp.py tests/test_gpu_c4.py tests/test_gpu_types_host.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_more.log 2>&1 || { tail -30 gpurun_out/pytest_more.log; exit 1; }
tail -1 gpurun_out/pytest_more.log
for n in 1000 4096 8192; do
  for lib in libeges_diag_prev.so libeges_diag.so; do
    EGES_DIAG_LIB=$lib timeout -k 10 100 python tools/phases.py $n > gpurun_out/ph_${n}_$lib.txt 2>&1
    echo "$lib $(grep launch gpurun_out/ph_${n}_$lib.txt)"
  done
done
cat gpurun_out/ph_1000_libeges_diag.so.txt | tail -9
for rep in 1 2; do
  timeout -k 10 200 python bench.py --config c3 --no-cpu-baseline > gpurun_out/c3_$rep.json 2> gpurun_out/c3.err
  python -c "import json;b=json.load(open('gpurun_out/c3_$rep.json'));print('c3', b['value'], b['p99_ms'], b['config']['correct'])"
done
