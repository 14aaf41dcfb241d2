# r02 first GPU pass: full GPU test suite (incl. C4 64M, logical devices, small grid), the default
# bench line, a kernel-trace profile of it and the PMC passes (pmc_traffic.json of these sources).
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --no-cpu-baseline > gpurun_out/prof.log 2>&1
bash tools/pmc.sh
cat gpurun_out/bench.json
tail -3 gpurun_out/pytest_gpu.log
