# Round-5 pass n: the lean row-form product / reduction (fr.cuh EGES_FR_LEAN=1: fewer instructions
# per product, the same values). Every GPU test on it, then a same-box alternating A/B against
# the EGES_FR_LEAN=0 build (libeges_base.so; native tools in tools/abbase/): C3 through bench.py
# (ctypes call + the kernel's HIP-event time), the native block caller, single calls.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r05_n
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for i in 1 2 3; do
  for lib in libeges_base.so libeges.so; do
    EGES_LIB=$lib timeout -k 10 200 python bench.py --config c3 --no-cpu-baseline > $O/c3_${lib%.so}_$i.json 2> $O/c3_${lib%.so}_$i.err
    python - "$O/c3_${lib%.so}_$i.json" "$lib" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print("c3", sys.argv[2], d["value"], d.get("p99_ms"), d.get("roofline", {}).get("kernel_ms"), d.get("config", {}).get("correct"))
PY
  done
  for b in tools/abbase/bin tools; do
    timeout -k 10 120 $b/block_bench 1000 300 > $O/bb_${b//\//_}_$i.json 2>&1
    timeout -k 10 120 $b/single_bench 1 3000 > $O/s1_${b//\//_}_$i.json 2>&1
    echo "$b block $(tail -1 $O/bb_${b//\//_}_$i.json)"
    echo "$b single $(tail -1 $O/s1_${b//\//_}_$i.json)"
  done
done
echo done rc=0
