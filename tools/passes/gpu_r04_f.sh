# Round-4 pass f: copies under a resident recover launch (blit kernel vs SDMA), and where a C3
# call's time goes outside its kernel (kernel + HIP API trace of tools/block_bench).
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04_f
mkdir -p $O
timeout -k 10 120 tools/copy_overlap_probe > $O/copy_overlap.json 2> $O/copy_overlap.err || { cat $O/copy_overlap.err; exit 1; }
cat $O/copy_overlap.json
for n in 1000 1; do
  timeout -k 10 200 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d $O/trace_bb_$n -o run -- tools/block_bench $n 200 > $O/trace_bb_$n.log 2>&1
  python tools/launch_gaps.py $O/trace_bb_$n
done
echo done rc=0
