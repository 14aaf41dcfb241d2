# tx_rows wave form: wire-format parity tests (both forms), C3 from wire bytes and C1.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_raw.py tests/test_gpu_rlp.py tests/test_gpu_block.py tests/test_gpu_types_host.py > gpurun_out/txrows_tests.log 2>&1
tail -2 gpurun_out/txrows_tests.log
timeout -k 10 200 python bench.py --config c3raw > gpurun_out/txrows_c3raw.json 2> gpurun_out/txrows_c3raw.err
timeout -k 10 200 python bench.py --config c1 > gpurun_out/txrows_c1.json 2> gpurun_out/txrows_c1.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3raw -o run --output-format csv -- python bench.py --config c3raw --no-cpu-baseline > gpurun_out/prof_c3raw.log 2>&1
head -c 300 gpurun_out/txrows_c3raw.json; echo; head -c 300 gpurun_out/txrows_c1.json; echo
python tools/kstats.py gpurun_out/prof_c3raw 2>/dev/null || find gpurun_out/prof_c3raw -name "*kernel_stats.csv" -exec head -5 {} \;
