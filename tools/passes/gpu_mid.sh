# Mid-size kernel bring-up: its parity tests, then the form curve (tools/formcurve.py).
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/mid_${1:-a}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_mid.py tests/test_c1.py -x -v --timeout 200 --timeout-method thread > $O/pytest_mid.log 2>&1 || { tail -40 $O/pytest_mid.log; exit 1; }
tail -3 $O/pytest_mid.log
timeout -k 10 400 python tools/formcurve.py ${2:-} > $O/formcurve.jsonl 2> $O/formcurve.err
cat $O/formcurve.jsonl
