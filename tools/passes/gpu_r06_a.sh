# Round-6 pass a: the publication probe (tools/publish_probe.hip) under every flag pattern and
# output memory type, then the default bench line as a box check.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r06_a
mkdir -p $O
P=tools/publish_probe
run() { timeout -k 10 120 $P "$@" >> $O/probe.jsonl 2>> $O/probe.err; tail -1 $O/probe.jsonl; }
run block default 40 1024 5 0
run block coherent 40 1024 5 0
run block noncoherent 40 1024 5 0
run block default 40 1024 5 2
run block default 40 1024 5 20
run sync default 20 1024 5 0
run last default 3000 64 2 0
run last coherent 3000 64 2 0
run last default 3000 64 2 5
run block default 40 1024 5 0 1
run block coherent 40 1024 5 0 1
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
cat $O/bench.json
echo done
