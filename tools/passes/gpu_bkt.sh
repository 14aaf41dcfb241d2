# Bucket-form mid kernel bring-up: its parity tests, then the form curve of both mid forms
# (tools/formcurve.py) and the stamped phases (tools/phases_mid.py; extra diag libs by suffix).
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/bkt_${1:-a}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_mid.py tests/test_gpu_exceptional.py tests/test_c1.py -x -v --timeout 200 --timeout-method thread > $O/pytest_mid.log 2>&1 || { tail -60 $O/pytest_mid.log; exit 1; }
tail -3 $O/pytest_mid.log
FORMCURVE_FORMS=${FORMS:-mid,midw} FORMCURVE_REPS=21 timeout -k 10 300 python tools/formcurve.py ${2:-2048,4096,10000,16384,24000,32768,50000} > $O/formcurve.jsonl 2> $O/formcurve.err
cat $O/formcurve.jsonl
EGES_MID_FORM=1 timeout -k 10 200 python tools/phases_mid.py 10000 > $O/phases_bkt.txt 2>&1
cat $O/phases_bkt.txt
for v in ${3:-}; do
  EGES_MID_FORM=1 EGES_DIAG_LIB=libeges_diag_$v.so timeout -k 10 200 python tools/phases_mid.py 10000 > $O/phases_bkt_$v.txt 2>&1
  echo "== variant $v"; cat $O/phases_bkt_$v.txt
done
