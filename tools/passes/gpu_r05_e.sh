# Round-5 pass e: the one-launch host-buffer form (run_host_one): its tests, then c2host with it
# and with the chunked path alternating; then the chunking-cost probes of pass d (device-resident
# 1M at EGES_GRID_MULT 1/2/4/8 and as 4 / 8 overlapped launches).
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r05_e
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_host_pipe.py tests/test_gpu_c4.py -x -v --timeout 200 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for i in 1 2 3; do
  for v in 1_4 1_1 1_8 0_4; do
    one=${v%_*}; fd=${v#*_}
    EGES_HOST_ONE=$one EGES_HOST_FEEDERS=$fd timeout -k 10 120 python bench.py --config c2host --steps 8 --warmup 2 > $O/c2host_${v}_$i.json 2>&1
    python -c "import json; a=json.load(open('$O/c2host_${v}_$i.json')); print('c2host one_feeders=$v', a['value'], a['ms_per_step'], a['fresh_outputs_sigs_per_s'], a['config']['correct'])"
  done
done
run() {  # name env...
  local name=$1; shift
  env "$@" timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-secondary --no-cpu-baseline --c4-total 0 > $O/$name.json 2> $O/$name.err
  python -c "import json; a=json.load(open('$O/$name.json')); print('$name', a['value'], a['roofline']['kernel_ms'], a['config']['correct'])"
}
for gm in 1 2 4 8; do run gm${gm} EGES_GRID_MULT=$gm; done
run ov4 EGES_OVERLAP=4
run ov8 EGES_OVERLAP=8
echo done rc=0
