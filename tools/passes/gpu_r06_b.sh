# Round-6 pass b: the publication probe under memory-system load (tools/publish_probe.hip, 8th
# argument): device-memory, host-read, host-write and all three at once.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r06_b
mkdir -p $O
P=tools/publish_probe
run() { timeout -k 10 120 $P "$@" >> $O/probe.jsonl 2>> $O/probe.err; tail -1 $O/probe.jsonl | cut -c1-420; }
for load in 1 2 3 4; do
  run block default 40 1024 5 0 4 $load
done
run block coherent 40 1024 5 0 4 4
run block default 40 1024 2 0 4 4
run block default 40 1024 10 0 4 4
run last default 2000 256 2 0 4 4
run last coherent 2000 256 2 0 4 4
run last default 400 1024 1 0 4 4
echo done
