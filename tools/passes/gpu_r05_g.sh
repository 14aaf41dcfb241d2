# Round-5 pass g: what the host-buffer path's chunking costs without any copies. Device-resident
# 1M at EGES_GRID_MULT 1/2/4/8 (8/4/2/1 signatures per thread) and the same 1M as 4 / 8 launches
# alternating two streams (EGES_OVERLAP), twice each.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r05_g
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
  run ov2_$i EGES_OVERLAP=2
done
echo done rc=0
