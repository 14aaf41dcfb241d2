# Round-6 pass k: (1) C1 with the one-per-CU bucket kernel compiled for two waves per SIMD
# (tools/abbk) against the product, alternating; (2) the two-per-CU bucket form against the
# one-per-CU one below 64 x CUs signatures (recovery, device-resident and sender rows; verify).
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r06_k
mkdir -p $O
for i in 1 2 3; do
  for v in prod abbk; do
    L=; [ $v = abbk ] && L=tools/abbk/libeges.so
    EGES_AB_LIB=$L timeout -k 10 200 python bench.py --config c1 --steps 40 > $O/c1_${v}_$i.json 2> $O/c1_${v}_$i.err
    python -c "import json; a=json.load(open('$O/c1_${v}_$i.json')); print('c1 $v', a['value'], a['ms_per_batch'], a['p99_ms'], a['config']['correct'], a['roofline']['kernel_ms'])"
  done
done
for i in 1 2; do
FORMCURVE_FORMS=mid,b2 FORMCURVE_REPS=15 timeout -k 10 300 python -u tools/formcurve.py 2000,4096,8192,10000,12000,16384 > $O/formcurve_$i.jsonl 2> $O/formcurve_$i.err || { tail -20 $O/formcurve_$i.err; exit 1; }
grep -v summary $O/formcurve_$i.jsonl | python -c "
import sys, json
for l in sys.stdin:
    r = json.loads(l); print(r['n'], r['form'], r['dev_ms'], r['whole_ms'], r['correct'])"
done
FORMCURVE_FORMS=bucket,b2 FORMCURVE_REPS=15 timeout -k 10 300 python -u tools/formcurve_verify.py 2000,4096,8192,12000,16384 > $O/formcurve_verify.jsonl 2> $O/formcurve_verify.err || { tail -20 $O/formcurve_verify.err; exit 1; }
grep -v summary $O/formcurve_verify.jsonl | cut -c1-160
echo done
