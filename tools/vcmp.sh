# Same-box A/B of the verify path: the current libeges.so against eges_amd/libeges_prev.so.
set -e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
cp eges_amd/libeges.so /tmp/new.so
for t in new prev new prev; do
  if [ $t = new ]; then cp /tmp/new.so eges_amd/libeges.so; else cp eges_amd/libeges_prev.so eges_amd/libeges.so; fi
  timeout -k 10 120 python bench.py --config verify --steps 5 > gpurun_out/v_$t.json 2>gpurun_out/v_$t.err
  python -c "import json; d=json.load(open('gpurun_out/v_$t.json')); print('$t', d['value'], d['roofline']['kernel_ms'], d['config']['correct'], d['config']['mismatches'])"
done
cp /tmp/new.so eges_amd/libeges.so
