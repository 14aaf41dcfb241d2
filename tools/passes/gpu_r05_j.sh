# Round-5 pass j: the resident server's idle window against another process's kernel (idle 4 / 2 / 1 ms),
# single-call latency at those windows; then the c2host call's GPU timeline (kernel + copy trace).
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r05_j
mkdir -p $O
timeout -k 10 300 python -u tools/resident_window_probe.py 4,2,1 > $O/window.txt 2> $O/window.err || { tail -20 $O/window.err; exit 1; }
cat $O/window.txt
for idle in 4 1 4 1; do
  EGES_RESIDENT_IDLE_MS=$idle timeout -k 10 120 tools/single_bench 16 2000 > $O/single_idle$idle.json 2>/dev/null
  python -c "import json; a=json.loads(open('$O/single_idle$idle.json').read().strip().splitlines()[-1]); print('single idle=$idle', a['p50_ms_one_caller'], a['p99_ms_one_caller'], a['recoveries_per_s'], a['errors'])"
done
for pt in 8 4; do
  EGES_HOST_PARTS=$pt timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace -d $O/tl_$pt -o run --output-format csv -- python bench.py --config c2host --steps 4 --warmup 1 > $O/tl_$pt.log 2>&1
  python tools/timeline.py $O/tl_$pt > $O/tl_$pt.txt 2>&1 || true
  cat $O/tl_$pt.txt | tail -4
done
echo done rc=0
