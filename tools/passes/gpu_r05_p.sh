# Round-5 pass p: fr.cuh EGES_FR_LEAN=2 with the fold's tail terms summed off the chain and row selects as
# a two-level tree (libeges.so, tools/) against the first LEAN=2 build (libeges_l2a.so, tools/abl2a/) Every GPU test on it, then a same-box
# and LEAN=0 (libeges_base.so, tools/abbase/); every GPU test first.

set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r05_p
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for i in 1 2 3; do
  for lib in libeges_base.so libeges_l2a.so libeges.so; do
    EGES_LIB=$lib timeout -k 10 200 python bench.py --config c3 --no-cpu-baseline > $O/c3_${lib%.so}_$i.json 2> $O/c3_${lib%.so}_$i.err
    python - "$O/c3_${lib%.so}_$i.json" "$lib" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print("c3", sys.argv[2], d["value"], d.get("p99_ms"), d.get("roofline", {}).get("kernel_ms"), d.get("config", {}).get("correct"))
PY
  done
  for b in tools/abbase/bin tools/abl2a/bin tools; do
    timeout -k 10 120 $b/block_bench 1000 300 > $O/bb_${b//\//_}_$i.json 2>&1
    timeout -k 10 120 $b/single_bench 1 3000 > $O/s1_${b//\//_}_$i.json 2>&1
    echo "$b block $(python -c "import json;d=json.loads(open('$O/bb_${b//\//_}_$i.json').read().strip().splitlines()[-1]);print(d['median_ms'],d['errors'])") single $(python -c "import json;d=json.loads(open('$O/s1_${b//\//_}_$i.json').read().strip().splitlines()[-1]);print(d['p50_ms_one_caller'],d['verify_p50_ms_one_caller'],d['errors'])")"
  done
done
echo done rc=0
