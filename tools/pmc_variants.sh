# One SQ counter pass + one TCC pass per libeges_<tag>.so variant (and the default build). Run via gpurun.
# Usage: bash tools/pmc_variants.sh tag1 tag2 ...
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
cp eges_amd/libeges.so /tmp/libeges_default.so
B="python bench.py --steps 2 --warmup 1 --no-cpu-baseline"
for tag in default "$@"; do
  if [ "$tag" = default ]; then cp /tmp/libeges_default.so eges_amd/libeges.so; else cp "eges_amd/libeges_$tag.so" eges_amd/libeges.so; fi
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_INT64 SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d "gpurun_out/pmcv_$tag" -o run --output-format csv -- $B > "gpurun_out/pmcv_$tag.log" 2>&1
  timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d "gpurun_out/pmcv_tcc_$tag" -o run --output-format csv -- $B > "gpurun_out/pmcv_tcc_$tag.log" 2>&1
done
cp /tmp/libeges_default.so eges_amd/libeges.so
echo done
