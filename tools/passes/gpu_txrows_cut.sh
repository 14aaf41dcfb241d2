# tx_rows cut check: wave form vs lane-serial form on C1-shaped batches just below the default cut
# (EGES_TXROWS_WAVE_MAX=0 forces the lane-serial form), alternating on one box.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for b in 2000 4096 8192; do
  for w in 0 1073741824 0 1073741824; do
    EGES_TXROWS_WAVE_MAX=$w timeout -k 10 200 python bench.py --config c1 --batch $b --no-cpu-baseline --steps 10 > gpurun_out/cut_c1_${b}_$w.json 2> gpurun_out/cut_c1_${b}_$w.err
    echo "c1 batch=$b wave_max=$w $(python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['unit'], d['ms_per_batch'], d['config']['correct'])" gpurun_out/cut_c1_${b}_$w.json)"
  done
done
