# Round-5 pass zb: where the windowed mid-size form stops paying (the routing curve showed 40,000
# signatures at 0.98 ms on it): windowed vs lane-serial vs two bucket generations around 32k
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r05_zb
FORMCURVE_FORMS=mid,midw,lane FORMCURVE_REPS=12 timeout -k 10 600 python -u tools/formcurve.py \
  20000,24000,28000,32768,36000,40000 | tee gpurun_out/r05_zb/formcurve_cut.jsonl
echo done rc=0
