# Round-6 pass l: the whole GPU suite on the bucket2 routing, then the product form curves from
# 1k to 131k (recovery: device-resident and C1-shaped wire calls; verify).
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r06_l
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
FORMCURVE_FORMS=auto FORMCURVE_REPS=10 timeout -k 10 500 python -u tools/formcurve.py 1000,1536,2000,4096,8192,10000,16384,16385,20000,24000,28000,32768,33000,40000,50000,65536,100000,131072 > $O/formcurve_auto.jsonl 2> $O/formcurve_auto.err || { tail -20 $O/formcurve_auto.err; exit 1; }
grep -v summary $O/formcurve_auto.jsonl | python -c "
import sys, json
for l in sys.stdin:
    r = json.loads(l); print(r['n'], r['form'], r['dev_ms'], r['whole_ms'], r['correct'])"
FORMCURVE_FORMS=auto FORMCURVE_REPS=10 timeout -k 10 500 python -u tools/formcurve_verify.py 1000,1536,2000,4096,8192,16384,20000,24000,32768,33000,40000,65536,100000,131072 > $O/formcurve_verify_auto.jsonl 2> $O/formcurve_verify_auto.err || { tail -20 $O/formcurve_verify_auto.err; exit 1; }
grep -v summary $O/formcurve_verify_auto.jsonl | cut -c1-130
echo done
