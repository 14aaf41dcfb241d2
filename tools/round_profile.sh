# End-of-milestone evidence on one GPU (run via gpurun): parity tests, smoke, the default bench
# line, kernel-trace profiles of it and of the C3 block bench, the PMC passes and every config.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
cat gpurun_out/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --no-cpu-baseline > gpurun_out/prof.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3 -o run --output-format csv -- python bench.py --config c3 --no-cpu-baseline > gpurun_out/prof_c3.log 2>&1
bash tools/pmc.sh
bash tools/passes/gpu_configs.sh
timeout -k 10 200 python bench.py --config c3raw > gpurun_out/bench_c3raw.json 2> gpurun_out/bench_c3raw.err
timeout -k 10 200 python bench.py --config c1 > gpurun_out/bench_c1.json 2> gpurun_out/bench_c1.err
timeout -k 10 200 tools/single_bench 8 2000 > gpurun_out/single.json 2> gpurun_out/single.err
timeout -k 10 200 tools/single_bench 16 2000 > gpurun_out/single16.json 2> gpurun_out/single16.err
ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1 timeout -k 10 300 tools/asan/sanitize_host 5000 > gpurun_out/sanitize_gpu.log 2>&1
cat gpurun_out/bench_c3raw.json gpurun_out/bench_c1.json gpurun_out/single.json gpurun_out/single16.json
tail -1 gpurun_out/sanitize_gpu.log
