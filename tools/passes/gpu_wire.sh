# Fused wire-format form (k_recover_mid.hip wire_stage / wire_parse): the wire-path parity tests
# (both forms), C1, then the form curve (fused / unfused bucket / windowed) and phases.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/wire_${1:-a}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_raw.py tests/test_gpu_rlp.py tests/test_gpu_block.py tests/test_c1.py tests/test_gpu_mid.py -x -v --timeout 200 --timeout-method thread > $O/pytest_wire.log 2>&1 || { tail -60 $O/pytest_wire.log; exit 1; }
tail -3 $O/pytest_wire.log
FORMCURVE_FORMS=${FORMS:-mid,midnf,midw} FORMCURVE_REPS=21 timeout -k 10 300 python tools/formcurve.py ${2:-4096,10000,16384} > $O/formcurve.jsonl 2> $O/formcurve.err
cat $O/formcurve.jsonl
timeout -k 10 200 python bench.py --config c1 --no-cpu-baseline > $O/bench_c1.json 2> $O/bench_c1.err
cat $O/bench_c1.json
