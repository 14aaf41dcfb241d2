# Round-4 pass c: host-buffer pipeline on one compute stream (chunk schedules, old path, 2-stream
# A/B), the lane-serial kernel by batch and grid generations, then the host-pipe tests and the
# host-code ASan harness on the GPU.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04_c
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_host_pipe.py -x -v --timeout 200 --timeout-method thread > $O/pytest_pipe.txt 2>&1 || { tail -30 $O/pytest_pipe.txt; exit 1; }
tail -1 $O/pytest_pipe.txt
c2h() {  # name env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --config c2host --steps 6 --warmup 2 > $O/c2host_$name.json 2> $O/c2host_$name.err
  python -c "import json; a=json.load(open('$O/c2host_$name.json')); print('c2host $name', a['value'], a['ms_per_step'], a['config']['correct'])"
}
for i in 1 2; do
  c2h default_$i EGES_HOST_PIPE=1
  c2h old_$i EGES_HOST_PIPE=0
  c2h f196_$i EGES_PIPE_FIRST=196608 EGES_PIPE_CHUNK=851968
  c2h f131_$i EGES_PIPE_FIRST=131072 EGES_PIPE_CHUNK=917504
  c2h f393_$i EGES_PIPE_FIRST=393216 EGES_PIPE_CHUNK=655360
  c2h f262x3_$i EGES_PIPE_FIRST=262144 EGES_PIPE_CHUNK=393216
  c2h two_$i EGES_PIPE_STREAMS=2
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c2host -o run --output-format csv -- python3 bench.py --config c2host --steps 3 --warmup 1 > $O/prof_c2host.log 2>&1
for gm in 1 2; do
  for b in 262144 393216 524288 786432 1048576; do
    EGES_GRID_MULT=$gm timeout -k 10 120 python bench.py --batch $b --steps 5 --warmup 2 --no-secondary --no-cpu-baseline > $O/gm${gm}_b$b.json 2> $O/gm${gm}_b$b.err
    python -c "import json; d=json.load(open('$O/gm${gm}_b$b.json')); print('grid_mult $gm batch $b kernel_ms', d['roofline']['kernel_ms'], d['config']['correct'])"
  done
done
ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1 timeout -k 10 300 tools/asan/sanitize_host 3000 > $O/sanitize_gpu.log 2>&1
tail -1 $O/sanitize_gpu.log
