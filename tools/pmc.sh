# PMC passes for the dominant kernels (one counter group per rocprofv3 run; each pass within the
# per-block limits: <= 8 SQ, FETCH_SIZE / WRITE_SIZE alone). Run via gpurun; writes
# gpurun_out/pmc_traffic.json in the schema bench.py reads (tools/pmc_summary.py).
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
B="python bench.py --steps 2 --warmup 1 --no-cpu-baseline"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY -d gpurun_out/pmc_sq -o run --output-format csv -- $B > gpurun_out/pmc_sq.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/pmc_sq2 -o run --output-format csv -- $B > gpurun_out/pmc_sq2.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- $B > gpurun_out/pmc_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- $B > gpurun_out/pmc_write.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pmc_tcc -o run --output-format csv -- $B > gpurun_out/pmc_tcc.log 2>&1
python tools/pmc_summary.py gpurun_out 1048576 gpurun_out/pmc_traffic.json > /dev/null
echo done
