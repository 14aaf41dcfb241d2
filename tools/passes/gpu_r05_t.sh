# Round-5 pass t: carry round 3 without the final lane mask (libeges.so, tools/) against the
# committed lean product (libeges_prev.so, tools/abprev/) and the round-4 code
# (libeges_base.so, tools/abbase/): every GPU
# test first, then a same-box alternating A/B (C3 kernel and call, native block caller, single calls).
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r05_t
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for i in 1 2 3; do
  for v in base:tools/abbase/bin prev:tools/abprev/bin :tools; do
    tag=${v%%:*}; b=${v#*:}; lib=libeges${tag:+_$tag}.so
    EGES_LIB=$lib timeout -k 10 200 python bench.py --config c3 --no-cpu-baseline > $O/c3_${tag:-final}_$i.json 2> $O/c3_${tag:-final}_$i.err
    timeout -k 10 120 $b/block_bench 1000 300 > $O/bb_${tag:-final}_$i.json 2>&1
    timeout -k 10 120 $b/single_bench 1 3000 > $O/s1_${tag:-final}_$i.json 2>&1
    python - $O ${tag:-final} $i <<'PY'
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
