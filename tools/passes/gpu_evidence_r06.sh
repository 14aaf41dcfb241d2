# Round-6 evidence on one GPU (via gpurun). Part "tests": every GPU test, smoke and the host-ASan
# harness. Part "perf": the default bench line, kernel stats of C2 / C1 / C3, the PMC passes
# (tools/pmc.sh), every bench config, the single-call and native C3 benches.
# Outputs under gpurun_out/ev6_TAG.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
PART=${1:-tests}
T=${2:-a}
O=gpurun_out/ev6_$T
mkdir -p $O
if [ "$PART" = tests ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
  tail -1 $O/pytest_gpu.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
  tail -1 $O/smoke.log
  ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1 timeout -k 10 300 tools/asan/sanitize_host 5000 > $O/sanitize_gpu.log 2>&1
  tail -1 $O/sanitize_gpu.log
  exit 0
fi
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
cat $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-secondary > $O/prof.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c1 -o run --output-format csv -- python3 bench.py --config c1 --no-cpu-baseline > $O/prof_c1.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c3 -o run --output-format csv -- python3 bench.py --config c3 --no-cpu-baseline > $O/prof_c3.log 2>&1
bash tools/pmc.sh > $O/pmc.log 2>&1
cp gpurun_out/pmc_traffic.json $O/
for cfg in c1 c3 c3raw; do
  timeout -k 10 200 python bench.py --config $cfg > $O/bench_$cfg.json 2> $O/bench_$cfg.err
  cat $O/bench_$cfg.json
done
for cfg in c5 verify c2host; do
  timeout -k 10 200 python bench.py --config $cfg --steps 5 > $O/bench_$cfg.json 2> $O/bench_$cfg.err
  cat $O/bench_$cfg.json
done
timeout -k 10 300 python bench.py --config c4 --steps 3 --warmup 1 > $O/bench_c4.json 2> $O/bench_c4.err
cat $O/bench_c4.json
timeout -k 10 300 python bench.py --config c4host --steps 2 --warmup 1 > $O/bench_c4host.json 2> $O/bench_c4host.err
cat $O/bench_c4host.json
timeout -k 10 200 tools/single_bench 8 2000 > $O/single8.json 2> $O/single8.err
timeout -k 10 200 tools/single_bench 16 2000 > $O/single16.json 2> $O/single16.err
cat $O/single8.json $O/single16.json
timeout -k 10 120 tools/block_bench 1000 300 > $O/block1000.json 2>&1
timeout -k 10 120 tools/block_bench 1 300 > $O/block1.json 2>&1
cat $O/block1000.json $O/block1.json
# the 16k-32k band on the two-per-CU bucket form: kernel stats of a 24,000-signature device-resident batch
FORMCURVE_FORMS=auto FORMCURVE_REPS=20 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_b2 -o run --output-format csv -- python3 tools/formcurve.py 24000 > $O/prof_b2.log 2>&1
echo done
