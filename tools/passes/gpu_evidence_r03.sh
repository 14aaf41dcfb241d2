# Round-3 evidence pass on one GPU (via gpurun): every GPU test, smoke, the default bench line,
# kernel stats of C2 / C1 / C3, the PMC passes (C2: tools/pmc.sh, C1: tools/pmc_c1.sh), every
# bench config, the single-call bench and the host-ASan harness. Outputs under gpurun_out/ev_TAG.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-a}
O=gpurun_out/ev_$T
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
cat $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-secondary > $O/prof.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c1 -o run --output-format csv -- python3 bench.py --config c1 --no-cpu-baseline > $O/prof_c1.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c3 -o run --output-format csv -- python3 bench.py --config c3 --no-cpu-baseline > $O/prof_c3.log 2>&1
bash tools/pmc.sh > $O/pmc.log 2>&1
cp gpurun_out/pmc_traffic.json $O/
bash tools/pmc_c1.sh > $O/pmc_c1.log 2>&1
cp gpurun_out/pmc_c1/pmc_c1.json $O/
for cfg in c1 c3 c3raw; do
  timeout -k 10 200 python bench.py --config $cfg > $O/bench_$cfg.json 2> $O/bench_$cfg.err
  cat $O/bench_$cfg.json
done
for cfg in c5 verify; do
  timeout -k 10 200 python bench.py --config $cfg --steps 3 > $O/bench_$cfg.json 2> $O/bench_$cfg.err
  cat $O/bench_$cfg.json
done
timeout -k 10 300 python bench.py --config c4 --steps 3 --warmup 1 > $O/bench_c4.json 2> $O/bench_c4.err
cat $O/bench_c4.json
timeout -k 10 200 tools/single_bench 8 2000 > $O/single8.json 2> $O/single8.err
timeout -k 10 200 tools/single_bench 16 2000 > $O/single16.json 2> $O/single16.err
cat $O/single8.json $O/single16.json
ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1 timeout -k 10 300 tools/asan/sanitize_host 5000 > $O/sanitize_gpu.log 2>&1
tail -1 $O/sanitize_gpu.log
