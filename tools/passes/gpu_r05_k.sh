# Round-5 pass k: host-buffer chunks through pinned staging (copy engine) instead of HIP's pageable
# copies (blit kernels), one or two compute streams: the host-pipe tests, then c2host A/B alternating,
# then the kernel + copy trace of the staged form.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r05_k
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_host_pipe.py -x -v --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for i in 1 2 3; do
  for v in 0_1_8 1_1_8 1_2_8 1_2_4 1_1_4; do
    IFS=_ read sg ss pt <<< "$v"
    EGES_HOST_STAGE=$sg EGES_HOST_STREAMS=$ss EGES_HOST_PARTS=$pt timeout -k 10 120 python bench.py --config c2host --steps 8 --warmup 2 > $O/c2host_${v}_$i.json 2> $O/c2host_${v}_$i.err
    python -c "import json; a=json.load(open('$O/c2host_${v}_$i.json')); print('c2host stage_streams_parts=$v', a['value'], a['ms_per_step'], a['fresh_outputs_sigs_per_s'], a['config']['correct'])"
  done
done
EGES_HOST_STAGE=1 EGES_HOST_STREAMS=2 timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace -d $O/tl_s2 -o run --output-format csv -- python bench.py --config c2host --steps 4 --warmup 1 > $O/tl_s2.log 2>&1
python tools/timeline.py $O/tl_s2 > $O/tl_s2.txt 2>&1 || true
tail -3 $O/tl_s2.txt
echo done rc=0
