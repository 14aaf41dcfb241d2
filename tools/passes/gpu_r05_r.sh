# Round-5 pass r: which of the LEAN=3 changes helps which latency form. Same box, alternating:
#   A libeges_l2a.so (LEAN=2 reduce, row-select chain, six-step normalize_weak)
#   B libeges.so     (LEAN=3 reduce, row-select tree, four-step normalize_weak)
#   C libeges_vc.so  (LEAN=3 reduce, chain, six-step)    D libeges_vd.so (LEAN=3 reduce, chain, four-step)
# C3 kernel (HIP events) and ctypes call, the native block caller, single recover / verify p50.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r05_r
mkdir -p $O
for i in 1 2 3; do
  for v in l2a:tools/abl2a/bin :tools vc:tools/abvc/bin vd:tools/abvd/bin; do
    tag=${v%%:*}; b=${v#*:}; lib=libeges${tag:+_$tag}.so
    EGES_LIB=$lib timeout -k 10 200 python bench.py --config c3 --no-cpu-baseline > $O/c3_${tag:-B}_$i.json 2> $O/c3_${tag:-B}_$i.err
    timeout -k 10 120 $b/block_bench 1000 300 > $O/bb_${tag:-B}_$i.json 2>&1
    timeout -k 10 120 $b/single_bench 1 3000 > $O/s1_${tag:-B}_$i.json 2>&1
    python - $O ${tag:-B} $i <<'PY'
import json, sys
o, t, i = sys.argv[1:]
last = lambda f: json.loads(open(f).read().strip().splitlines()[-1])
c3, bb, s1 = last(f"{o}/c3_{t}_{i}.json"), last(f"{o}/bb_{t}_{i}.json"), last(f"{o}/s1_{t}_{i}.json")
print(t, i, "c3", c3["value"], c3["roofline"]["kernel_ms"], c3["config"]["correct"], "native", bb["median_ms"], bb["errors"],
      "single", s1["p50_ms_one_caller"], s1["verify_p50_ms_one_caller"], s1["errors"])
PY
  done
done
echo done rc=0
