# Round-6 pass j: the two-per-CU bucket form (EGES_BKT2): its tests, then recovery and verify
# form curves in the 16k-40k band, the new routing (auto) against round 5's (auto_nob2).
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r06_j
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_mid.py tests/test_gpu_exceptional.py tests/test_gpu_handoff.py tests/test_gpu_verify_mid.py tests/test_gpu_sender_fused.py tests/test_gpu_gate.py > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
FORMCURVE_FORMS=auto,auto_nob2,b2 FORMCURVE_REPS=10 timeout -k 10 400 python -u tools/formcurve.py 10000,16384,16385,20000,24000,28000,32768,33000,40000,65536 > $O/formcurve.jsonl 2> $O/formcurve.err || { tail -20 $O/formcurve.err; exit 1; }
grep -v summary $O/formcurve.jsonl | python -c "
import sys, json
for l in sys.stdin:
    r = json.loads(l); print(r['n'], r['form'], r['dev_ms'], r['whole_ms'], r['correct'])"
FORMCURVE_FORMS=auto,auto_nob2 FORMCURVE_REPS=10 timeout -k 10 400 python -u tools/formcurve_verify.py 10000,16384,20000,24000,32768,40000 > $O/formcurve_verify.jsonl 2> $O/formcurve_verify.err || { tail -20 $O/formcurve_verify.err; exit 1; }
grep -v summary $O/formcurve_verify.jsonl | cut -c1-200
echo done
