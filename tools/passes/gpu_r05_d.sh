# Round-5 pass d: what the host-buffer path's chunking costs without any copies. Device-resident
# 1M: lane-serial generations (EGES_GRID_MULT 1/2/4/8, i.e. 8/4/2/1 signatures per thread) and
# the same 1M split into 4 / 8 launches alternating two streams (EGES_OVERLAP); the c2host line.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r05_d
mkdir -p $O
run() {  # name env...
  local name=$1; shift
  env "$@" timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-secondary --no-cpu-baseline --c4-total 0 > $O/$name.json 2> $O/$name.err
  python -c "import json; a=json.load(open('$O/$name.json')); print('$name', a['value'], a['roofline']['kernel_ms'], a['config']['correct'])"
}
for i in 1 2; do
  for gm in 1 2 4 8; do run gm${gm}_$i EGES_GRID_MULT=$gm; done
  run ov4_$i EGES_OVERLAP=4
  run ov8_$i EGES_OVERLAP=8
done
for i in 1 2; do
  timeout -k 10 120 python bench.py --config c2host --steps 8 --warmup 2 > $O/c2host_$i.json 2>&1
  python -c "import json; a=json.load(open('$O/c2host_$i.json')); print('c2host', a['value'], a['ms_per_step'])"
done
echo done rc=0
