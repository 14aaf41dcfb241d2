# Round-4 pass u: EGES_GATE=2 (wire-format calls on the latency kernels gated too): the gate / wire
# tests with it, then C3 from wire bytes (bench, ctypes caller) with EGES_GATE 1 and 2, alternating.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04_u
mkdir -p $O
EGES_GATE=2 timeout -k 10 400 python -u -m pytest tests/test_gpu_gate.py tests/test_gpu_raw.py tests/test_gpu_block.py tests/test_gpu_handoff.py -x -v --timeout 250 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -60 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for i in 1 2 3; do
  for g in 2 1; do
    EGES_GATE=$g timeout -k 10 200 python bench.py --config c3raw --no-cpu-baseline > $O/c3raw_g${g}_$i.json 2> $O/c3raw_g${g}_$i.err
    python -c "import json; a=json.load(open('$O/c3raw_g${g}_$i.json')); print('gate $g c3raw', a['value'], a['p99_ms'])"
  done
done
echo done rc=0
