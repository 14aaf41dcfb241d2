# Round-5 pass za: the product routing's curve from 1 to 1M signatures (tools/formcurve.py, form
# "auto"): C1-shaped wire-format calls through eges_sender_raw_batch and device-resident launches
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r05_za
FORMCURVE_FORMS=auto FORMCURVE_REPS=12 timeout -k 10 600 python -u tools/formcurve.py \
  1,16,100,256,448,1000,1536,2000,4096,10000,16384,24000,40000,65536,131072,262144,1048576 \
  | tee gpurun_out/r05_za/formcurve_auto.jsonl
echo done rc=0
