# End-of-milestone evidence on one GPU (run via gpurun): parity tests, the default bench line,
# a kernel-trace profile of the same command, the PMC passes and every bench config.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --no-cpu-baseline > gpurun_out/prof.log 2>&1
bash tools/pmc.sh
bash tools/gpu_configs.sh
timeout -k 10 200 python bench.py --config c3raw > gpurun_out/bench_c3raw.json 2> gpurun_out/bench_c3raw.err
cat gpurun_out/bench.json gpurun_out/bench_c3raw.json
tail -1 gpurun_out/pytest_gpu.log
