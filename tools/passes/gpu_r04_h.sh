# Round-4 pass h: the host-buffer pipeline with segment-overlapped copies / DMA against the chunked
# path, and where C1's call time goes outside its kernel.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04_h
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_host_pipe.py -x -v --timeout 200 --timeout-method thread > $O/pytest_pipe.txt 2>&1 || { tail -30 $O/pytest_pipe.txt; exit 1; }
tail -1 $O/pytest_pipe.txt
c2h() {  # name env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --config c2host --steps 8 --warmup 2 > $O/c2host_$name.json 2> $O/c2host_$name.err
  python -c "import json; a=json.load(open('$O/c2host_$name.json')); print('c2host $name', a['value'], a['ms_per_step'], a['fresh_outputs_sigs_per_s'], a['config']['correct'])"
}
for i in 1 2; do
  c2h pipe_262_786_$i EGES_HOST_PIPE=1
  c2h pipe_262x4_$i EGES_HOST_PIPE=1 EGES_PIPE_FIRST=262144 EGES_PIPE_CHUNK=262144
  c2h pipe_131_459_$i EGES_HOST_PIPE=1 EGES_PIPE_FIRST=131072 EGES_PIPE_CHUNK=458752
  c2h pipe_131_917_$i EGES_HOST_PIPE=1 EGES_PIPE_FIRST=131072 EGES_PIPE_CHUNK=917504
  c2h pipe_262_786_s4_$i EGES_HOST_PIPE=1 EGES_PIPE_SEG=4194304
  c2h parts4_$i EGES_HOST_PIPE=0 EGES_HOST_PARTS=4
  c2h parts8_$i EGES_HOST_PIPE=0 EGES_HOST_PARTS=8
done
EGES_AB_LIB=$PWD/eges_amd/libeges_diag.so timeout -k 10 120 python tools/c1_host_phases.py 10000 100 > $O/c1_phases.json 2> $O/c1_phases.err
cat $O/c1_phases.json
timeout -k 10 200 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d $O/trace_c1 -o run -- python3 tools/c1_host_phases.py 10000 100 > $O/trace_c1.log 2>&1
python tools/launch_gaps.py $O/trace_c1 recover_bkt_kernel
bb() {  # name n env...
  local name=$1 n=$2; shift 2
  env "$@" timeout -k 10 120 tools/block_bench $n 200 > $O/bb_${name}.json 2>&1
  python -c "import json; a=json.load(open('$O/bb_${name}.json')); print('bb $name', a['median_ms'], a['p99_ms'], a['errors'])"
}
for n in 1 16 64 128 256 320 384 448 512; do
  bb split_$n $n EGES_LAT_WIDE_MAX=100000
  bb tri_$n $n EGES_LAT_WIDE_MAX=0 EGES_LAT_TRI_MAX=100000
  bb narrow_$n $n EGES_LAT_WIDE_MAX=0 EGES_LAT_TRI_MAX=0
done
echo done rc=0
