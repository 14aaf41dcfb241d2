# Staged latency-kernel inputs (sender.cuh stage_inputs): parity suites, then same-box A/B
# against the base build: C3 (sender rows, host buffers) and the single-call entries.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/stage_${1:-a}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_lat.py tests/test_gpu_mid.py tests/test_gpu_types_host.py tests/test_gpu_block.py tests/test_gpu_concurrency.py tests/test_gpu_exceptional.py -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for i in 1 2 3; do
  for lib in libeges_base.so libeges.so; do
    EGES_LIB=$lib timeout -k 10 200 python bench.py --config c3 --no-cpu-baseline > $O/c3_${lib%.so}_$i.json 2> $O/c3_${lib%.so}_$i.err
    echo "c3 $lib run $i: $(python -c "import json;d=json.load(open('$O/c3_${lib%.so}_$i.json'));print(d['value'], d['unit'], d.get('p99_ms'))")"
  done
  LD_LIBRARY_PATH=$PWD/tools/abbase timeout -k 10 120 tools/single_bench 8 2000 > $O/single_base_$i.json 2> $O/single_base_$i.err
  timeout -k 10 120 tools/single_bench 8 2000 > $O/single_new_$i.json 2> $O/single_new_$i.err
  echo "single base $i: $(cat $O/single_base_$i.json | cut -c1-200)"
  echo "single new  $i: $(cat $O/single_new_$i.json | cut -c1-200)"
done
