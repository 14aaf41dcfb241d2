# Wave Keccak A/B (eges_amd/libeges_diag_prev.so: the diagnostic build of the previous form, built
# by hand, e.g. -DEGES_KECCAK_HALVES=0; earlier the dropped two-step round vs the four-step one): parity tests of every path that ends in a
# wave Keccak, then stamped launches at n = 1 / 1000 alternating, C3 and C3 from wire bytes.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_lat.py tests/test_gpu_parity.py tests/test_gpu_raw.py tests/test_gpu_rlp.py tests/test_gpu_block.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_kw.log 2>&1 || { tail -30 gpurun_out/pytest_kw.log; exit 1; }
tail -1 gpurun_out/pytest_kw.log
for n in 1 1000; do
  for lib in libeges_diag_prev.so libeges_diag.so libeges_diag_prev.so libeges_diag.so; do
    EGES_DIAG_LIB=$lib timeout -k 10 100 python tools/phases.py $n > gpurun_out/kw_${n}_$lib.txt 2>&1
    echo "n=$n $lib $(grep launch gpurun_out/kw_${n}_$lib.txt) $(grep -i keccak gpurun_out/kw_${n}_$lib.txt)"
  done
done
timeout -k 10 200 python bench.py --config c3 --no-cpu-baseline > gpurun_out/kw_c3.json 2> gpurun_out/kw_c3.err
timeout -k 10 200 python bench.py --config c3raw --no-cpu-baseline > gpurun_out/kw_c3raw.json 2> gpurun_out/kw_c3raw.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_kw -o run --output-format csv -- python bench.py --config c3raw --no-cpu-baseline > gpurun_out/prof_kw.log 2>&1
head -c 200 gpurun_out/kw_c3.json; echo; head -c 200 gpurun_out/kw_c3raw.json; echo
python -c "import csv; [print(r['Name'][:40], r['Calls'], r['AverageNs']) for r in csv.DictReader(open('gpurun_out/prof_kw/run_kernel_stats.csv'))]" 
