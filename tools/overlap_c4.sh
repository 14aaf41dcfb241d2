# Same-box A/B of EGES_OVERLAP on configs[3] (64M signatures, every address checked). Run via gpurun.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do
  for s in 0 2; do
    EGES_OVERLAP=$s timeout -k 10 200 python bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/ovc4_${s}_${rep}.json 2> gpurun_out/ovc4_${s}_${rep}.err
    echo "c4 overlap=$s rep=$rep $(python -c "import json;d=json.load(open('gpurun_out/ovc4_${s}_${rep}.json'));print(d['value'],d['ms_per_step'],d['config']['correct'])")"
  done
done
