# Round-6 pass w: the bucket form's wire stage issues every load of a thread before its first LDS
# store (one bus round trip). Wire tests, then same-box A/B against the previous build
# (tools/abst): C1 (bench.py --config c1) alternating.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06_w
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_c1.py tests/test_gpu_raw.py tests/test_gpu_gate.py tests/test_gpu_mid.py tests/test_gpu_handoff.py > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for i in 1 2 3 4; do
  for v in new old; do
    L=; [ $v = old ] && L=tools/abst/libeges.so
    EGES_AB_LIB=$L timeout -k 10 200 python bench.py --config c1 --no-cpu-baseline > $O/c1_${v}_$i.json 2> $O/c1_${v}_$i.err
    python -c "
import json; r=json.load(open('$O/c1_${v}_$i.json'))
print('$v', r.get('ms_per_batch'), r['roofline'].get('kernel_ms'), r['config']['correct'])"
  done
done
echo done
