# Recover-kernel cut check (EGES_LAT_MAX, read per call): latency kernel vs lane-serial kernel on
# C1-shaped batches between 2000 and 8192, alternating on one box.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for b in 2000 3000 4096 6000 8192; do
  for m in 0 8192 0 8192; do
    EGES_LAT_MAX=$m timeout -k 10 200 python bench.py --config c1 --batch $b --no-cpu-baseline --steps 10 > gpurun_out/latcut_${b}_$m.json 2> gpurun_out/latcut_${b}_$m.err
    echo "c1 batch=$b lat_max=$m $(python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['unit'], d['ms_per_batch'], d['config']['correct'])" gpurun_out/latcut_${b}_$m.json)"
  done
done
