# Same-box A/B of EGES_OVERLAP (overlapped recover launches on two streams). Run via gpurun.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do
  for s in 0 2 3 4; do
    EGES_OVERLAP=$s timeout -k 10 120 python bench.py --steps 8 --no-cpu-baseline > gpurun_out/ov_${s}_${rep}.json 2> gpurun_out/ov_${s}_${rep}.err
    echo "overlap=$s rep=$rep $(python -c "import json;d=json.load(open('gpurun_out/ov_${s}_${rep}.json'));print(d['value'],d['ms_per_step'],d['config']['correct'])")"
  done
done
