# PMC passes of the C1 bench (10k wire-format transfers: the fused bucket form of the mid-size
# kernel), one counter group per rocprofv3 run within the per-block limits.
# Writes gpurun_out/pmc_c1/pmc_c1.json.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_c1
B="python bench.py --config c1 --steps 5 --warmup 1 --no-cpu-baseline"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_WAVES SQ_WAIT_INST_ANY -d gpurun_out/pmc_c1/pmc_sq -o run --output-format csv -- $B > gpurun_out/pmc_c1/sq.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_ACTIVE_INST_SALU SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_INT64 -d gpurun_out/pmc_c1/pmc_sq2 -o run --output-format csv -- $B > gpurun_out/pmc_c1/sq2.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_c1/pmc_fetch -o run --output-format csv -- $B > gpurun_out/pmc_c1/fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_c1/pmc_write -o run --output-format csv -- $B > gpurun_out/pmc_c1/write.log 2>&1
python - <<'PY'
import json, sys
sys.path.insert(0, "tools")
from pmc_summary import summarise
s = summarise("gpurun_out/pmc_c1")
json.dump(s, open("gpurun_out/pmc_c1/pmc_c1.json", "w"), indent=1)
print(json.dumps(s.get("eges::recover_bkt_kernel", {}), indent=1))
PY
