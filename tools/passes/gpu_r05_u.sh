# Round-5 pass u: two more depth cuts in the row-form product, same box, alternating:
#   cur  libeges.so     (committed)
#   s    libeges_s.so   (EGES_FR_SPLIT3: each MAD chain's sum split on its own, no 64-bit merges)
#   e    libeges_e.so   (EGES_FR_EARLY16: column 16's product split before its carries arrive)
#   se   libeges_se.so  (both)
# C3 kernel (HIP events) and ctypes call (every address checked), native block caller, single calls.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r05_u
mkdir -p $O
for i in 1 2 3; do
  for v in :tools s:tools/abs/bin e:tools/abe/bin se:tools/abse/bin; do
    tag=${v%%:*}; b=${v#*:}; lib=libeges${tag:+_$tag}.so
    EGES_LIB=$lib timeout -k 10 200 python bench.py --config c3 --no-cpu-baseline > $O/c3_${tag:-cur}_$i.json 2> $O/c3_${tag:-cur}_$i.err
    timeout -k 10 120 $b/block_bench 1000 300 > $O/bb_${tag:-cur}_$i.json 2>&1
    timeout -k 10 120 $b/single_bench 1 3000 > $O/s1_${tag:-cur}_$i.json 2>&1
    python - $O ${tag:-cur} $i <<'PY'
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
