# C1 iteration (bucket form): mid / exceptional / wire parity tests, C1 bench x3, phases of the
# device-resident and the wire-format (fused) paths.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/c1x_${1:-a}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_mid.py tests/test_gpu_exceptional.py tests/test_gpu_raw.py tests/test_gpu_block.py tests/test_c1.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2 3; do timeout -k 10 200 python bench.py --config c1 --no-cpu-baseline > $O/c1_$i.json 2>> $O/c1.err; python -c "import json; d=json.load(open('$O/c1_$i.json')); print('c1', d['ms_per_batch'], d['p99_ms'])"; done
timeout -k 10 200 python tools/phases_mid.py 10000 > $O/phases.txt 2>&1
cat $O/phases.txt
PHASES_WIRE=1 timeout -k 10 200 python tools/phases_mid.py 10000 > $O/phases_wire.txt 2>&1
cat $O/phases_wire.txt
