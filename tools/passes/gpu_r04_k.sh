# Round-4 pass k: the chunked host path with its kernels on two alternating compute streams
# (EGES_HOST_STREAMS) against one, by chunk count, alternating.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04_k
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_host_pipe.py -x -v --timeout 200 --timeout-method thread > $O/pytest_pipe.txt 2>&1 || { tail -30 $O/pytest_pipe.txt; exit 1; }
tail -1 $O/pytest_pipe.txt
c2h() {  # name env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --config c2host --steps 8 --warmup 2 > $O/c2host_$name.json 2> $O/c2host_$name.err
  python -c "import json; a=json.load(open('$O/c2host_$name.json')); print('c2host $name', a['value'], a['ms_per_step'], a['fresh_outputs_sigs_per_s'], a['config']['correct'])"
}
for i in 1 2; do
  for p in 4 8; do
    c2h p${p}_s1_$i EGES_HOST_PARTS=$p EGES_HOST_STREAMS=1
    c2h p${p}_s2_$i EGES_HOST_PARTS=$p EGES_HOST_STREAMS=2
  done
done
echo done rc=0
