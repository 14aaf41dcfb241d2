# A/B of EGES_GRID_MULT (recover grid = k resident grids) on C2 and C4, alternating, one box.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for rep in ${REPS:-1 2}; do
  for m in ${MULTS:-1 2}; do
    EGES_GRID_MULT=$m timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 > gpurun_out/gm_${m}_$rep.json 2> gpurun_out/gm.err
    python -c "import json;b=json.load(open('gpurun_out/gm_${m}_$rep.json'));print('mult=$m rep=$rep', b['value'], b['roofline']['kernel_ms'], b['config']['correct'])"
  done
done
for m in ${C4MULTS:-1 2}; do
  EGES_GRID_MULT=$m timeout -k 10 300 python bench.py --config c4 --no-cpu-baseline > gpurun_out/gm_c4_$m.json 2>> gpurun_out/gm.err
  python -c "import json;b=json.load(open('gpurun_out/gm_c4_$m.json'));print('c4 mult=$m', b['value'], b['config']['correct'])"
done
