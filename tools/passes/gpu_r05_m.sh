# Round-5 pass m: the bucket form's verify mode over two generations of workgroups
# (EGES_VERIFY_MID_GENS): its tests, then the verify form curve across the 16k-65k band.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r05_m
timeout -k 10 300 python -u -m pytest tests/test_gpu_verify_mid.py -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/r05_m/pytest.txt 2>&1
tail -3 gpurun_out/r05_m/pytest.txt
FORMCURVE_FORMS=auto,auto2,lane FORMCURVE_REPS=10 timeout -k 10 300 python -u tools/formcurve_verify.py \
  12000,16384,20000,24000,28000,32000,40000,65536 > gpurun_out/r05_m/formcurve_verify.jsonl 2> gpurun_out/r05_m/formcurve.err
python - <<'PY'
import json
for l in open("gpurun_out/r05_m/formcurve_verify.jsonl"):
    try:
        d = json.loads(l)
    except Exception:
        continue
    if "n" in d:
        print(d["n"], d["form"], d.get("dev_ms"), d.get("whole_ms"), d.get("correct"))
PY
echo done rc=0
