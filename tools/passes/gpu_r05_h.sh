# Round-5 pass h: the progressive gate (EGES_GATE_STEP): gate / C1 / mid-size tests, then C1 with
# pieces of 16 workgroups against one piece, alternating (native-caller-free: bench --config c1);
# then what the host-buffer path's chunking costs without copies (device-resident 1M at
# EGES_GRID_MULT 1/2/4/8 and as 2 / 4 / 8 overlapped launches).
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r05_h
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_gate.py tests/test_c1.py tests/test_gpu_mid.py tests/test_gpu_handoff.py -x -v --timeout 200 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for i in 1 2 3; do
  for st in 16 0 8; do
    EGES_GATE_STEP=$st timeout -k 10 120 python bench.py --config c1 --steps 10 --warmup 3 --no-cpu-baseline > $O/c1_step${st}_$i.json 2> $O/c1_step${st}_$i.err
    python -c "import json; a=json.load(open('$O/c1_step${st}_$i.json')); print('c1 step=$st', a['ms_per_batch'], a['p99_ms'], a['roofline']['kernel_ms'], a['config']['correct'])"
  done
done
for i in 1 2; do
  for v in 8_0 4_1 4_0 2_1; do
    IFS=_ read pt gs <<< "$v"
    EGES_HOST_PARTS=$pt EGES_HOST_GENS=$gs timeout -k 10 120 python bench.py --config c2host --steps 8 --warmup 2 > $O/c2host_${v}_$i.json 2> $O/c2host_${v}_$i.err
    python -c "import json; a=json.load(open('$O/c2host_${v}_$i.json')); print('c2host parts_gens=$v', a['value'], a['ms_per_step'], a['config']['correct'])"
  done
done
run() {  # name env...
  local name=$1; shift
  env "$@" timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-secondary --no-cpu-baseline --c4-total 0 > $O/$name.json 2> $O/$name.err
  python -c "import json; a=json.load(open('$O/$name.json')); print('$name', a['value'], a['roofline']['kernel_ms'], a['config']['correct'])"
}
for gm in 1 2 4 8; do run gm${gm} EGES_GRID_MULT=$gm; done
for ov in 2 4 8; do run ov${ov} EGES_OVERLAP=$ov; done
echo done rc=0
