# Hoisted additions in the latency kernels' Strauss windows (frg.cuh gejq_double_pre /
# gejq_add_pre): latency-path parity suites, phases at n = 1000 and 16, then same-box A/B
# against the base build (C3, C3 from wire bytes, single calls).
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/hoist_${1:-a}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_lat.py tests/test_gpu_parity.py tests/test_gpu_exceptional.py tests/test_gpu_concurrency.py tests/test_gpu_raw.py -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
EGES_LAT_WIDE_MAX=0 timeout -k 10 120 python tools/phases.py 1000 > $O/phases_n1000.txt 2>&1
timeout -k 10 120 python tools/phases.py 16 > $O/phases_n16.txt 2>&1
head -12 $O/phases_n1000.txt
for i in 1 2 3; do
  for cfg in c3 c3raw; do
    for lib in libeges_base.so libeges.so; do
      EGES_LIB=$lib timeout -k 10 200 python bench.py --config $cfg --no-cpu-baseline > $O/${cfg}_${lib%.so}_$i.json 2> $O/${cfg}_${lib%.so}_$i.err
      echo "$cfg $lib run $i: $(python -c "import json;d=json.load(open('$O/${cfg}_${lib%.so}_$i.json'));print(d['value'], d['unit'], d.get('p99_ms'))")"
    done
  done
  LD_LIBRARY_PATH=$PWD/tools/abbase timeout -k 10 120 tools/single_bench 8 2000 > $O/single_base_$i.json 2> $O/single_base_$i.err
  timeout -k 10 120 tools/single_bench 8 2000 > $O/single_new_$i.json 2> $O/single_new_$i.err
  echo "single base $i: $(cut -c1-150 $O/single_base_$i.json)"
  echo "single new  $i: $(cut -c1-150 $O/single_new_$i.json)"
done
