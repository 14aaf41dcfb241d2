# Round-4 pass d: c2host with reused output arrays (no first-touch faults inside the call):
# pipelined schedules against the old chunked path.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04_d
mkdir -p $O
c2h() {  # name env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --config c2host --steps 8 --warmup 2 > $O/c2host_$name.json 2> $O/c2host_$name.err
  python -c "import json; a=json.load(open('$O/c2host_$name.json')); print('c2host $name', a['value'], a['ms_per_step'], a['fresh_outputs_sigs_per_s'], a['config']['correct'])"
}
for i in 1 2; do
  c2h default_$i EGES_HOST_PIPE=1
  c2h old_$i EGES_HOST_PIPE=0
  c2h f131_$i EGES_PIPE_FIRST=131072 EGES_PIPE_CHUNK=917504
  c2h f196_$i EGES_PIPE_FIRST=196608 EGES_PIPE_CHUNK=851968
  c2h f65_$i EGES_PIPE_FIRST=65536 EGES_PIPE_CHUNK=983040
done
EGES_HOST_PIPE=0 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $O/prof_old -o run --output-format csv -- python3 bench.py --config c2host --steps 3 --warmup 1 > $O/prof_old.log 2>&1
echo done rc=0
