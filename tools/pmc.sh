# PMC passes of the three measured kernels, one counter group per rocprofv3 run (within the
# per-block limits: <= 8 SQ, FETCH_SIZE / WRITE_SIZE alone), each config in its own process so
# every entry holds one kernel at one launch size:
#   c2: recover_kernel on 1,048,576 signatures (bench.py default line, no secondaries)
#   c3: recover_lat_kernel on a 1000-transaction block (bench.py --config c3)
#   c1: recover_bkt_kernel on 10,000 wire-format transfers (bench.py --config c1)
# Run via gpurun; writes gpurun_out/pmc_traffic.json in the schema bench.py reads
# (tools/pmc_summary.py).
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
G1="SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY"
G2="SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
for cfg in c2 c3 c1; do
  case $cfg in
    c2) B="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-secondary" ;;
    c3) B="python3 bench.py --config c3 --steps 1 --warmup 1 --no-cpu-baseline" ;;
    c1) B="python3 bench.py --config c1 --steps 1 --warmup 1 --no-cpu-baseline" ;;
  esac
  D=gpurun_out/pmc_$cfg
  mkdir -p $D
  timeout -s KILL 150 rocprofv3 --pmc $G1 -d $D/pmc_sq -o run --output-format csv -- $B > $D/sq.log 2>&1
  timeout -s KILL 150 rocprofv3 --pmc $G2 -d $D/pmc_sq2 -o run --output-format csv -- $B > $D/sq2.log 2>&1
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $D/pmc_fetch -o run --output-format csv -- $B > $D/fetch.log 2>&1
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $D/pmc_write -o run --output-format csv -- $B > $D/write.log 2>&1
  timeout -s KILL 150 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $D/pmc_tcc -o run --output-format csv -- $B > $D/tcc.log 2>&1
  echo "pmc $cfg done"
done
python3 tools/pmc_summary.py gpurun_out/pmc_traffic.json c2:eges::recover_kernel:1048576:gpurun_out/pmc_c2 \
  c3:eges::recover_lat_kernel:1000:gpurun_out/pmc_c3 c1:eges::recover_bkt_kernel:10000:gpurun_out/pmc_c1 > /dev/null
echo done
