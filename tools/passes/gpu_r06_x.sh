# Round-6 pass x: the bucket form folds u1 G into the first GLV half's bucket B1 on E' (wave S,
# an exact join after Y1's last add), so Y1's tail has one join less. The bucket-form tests, then
# same-box A/B against the previous build (tools/abg): C1, and device-resident recovery / verify
# form curves at 8k / 20k / 32k, alternating.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06_x
mkdir -p $O
[ -n "$SKIP_TESTS" ] || timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_exceptional.py tests/test_gpu_mid.py tests/test_gpu_verify_mid.py tests/test_gpu_handoff.py tests/test_gpu_gate.py tests/test_c1.py tests/test_gpu_routing.py tests/test_gpu_sender_fused.py tests/test_gpu_concurrency.py > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
[ -n "$SKIP_TESTS" ] || tail -1 $O/pytest.txt
for i in 1 2 3; do
  for v in new old; do
    L=; [ $v = old ] && L=tools/abg/libeges.so
    EGES_AB_LIB=$L timeout -k 10 200 python bench.py --config c1 --no-cpu-baseline > $O/c1_${v}_$i.json 2> $O/c1_${v}_$i.err
    EGES_AB_LIB=$L FORMCURVE_FORMS=auto FORMCURVE_REPS=20 timeout -k 10 200 python tools/formcurve.py 8192,20000,32768 > $O/fc_${v}_$i.jsonl 2> $O/fc_${v}_$i.err
    EGES_AB_LIB=$L FORMCURVE_FORMS=auto FORMCURVE_REPS=20 timeout -k 10 200 python tools/formcurve_verify.py 8192,20000,32768 > $O/fcv_${v}_$i.jsonl 2> $O/fcv_${v}_$i.err
    python -c "
import json
c=json.load(open('$O/c1_${v}_$i.json'))
f=[json.loads(l) for l in open('$O/fc_${v}_$i.jsonl') if '"n"' in l]
g=[json.loads(l) for l in open('$O/fcv_${v}_$i.jsonl') if '"n"' in l]
print('$v', 'c1', c.get('ms_per_batch'), c['roofline'].get('kernel_ms'), 'rec', [(d['n'], d.get('dev_ms')) for d in f], 'ver', [(d['n'], d.get('dev_ms')) for d in g])"
  done
done
echo done
