# Sender rows classified inside the latency / mid-size kernels (sender.cuh item_parse): the
# sender-path parity suites, then C3 (eges_sender_batch, host buffers) and C1 whole-call timings
# and C3's kernel list.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/snd_${1:-a}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_lat.py tests/test_gpu_mid.py tests/test_gpu_types_host.py tests/test_gpu_block.py -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --config c3 --no-cpu-baseline > $O/c3_$i.json 2> $O/c3_$i.err
  timeout -k 10 200 python bench.py --config c1 --no-cpu-baseline > $O/c1_$i.json 2> $O/c1_$i.err
  echo "run $i: c3 $(python -c "import json;print(json.load(open('$O/c3_$i.json'))['value'])") ms, c1 $(python -c "import json;d=json.load(open('$O/c1_$i.json'));print(d['value'], d.get('ms_per_call', d.get('p50_ms')))")"
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o c3 -- python bench.py --config c3 --no-cpu-baseline > $O/c3_prof.json 2> $O/c3_prof.err
find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats_c3.csv \;
cut -c1-120 $O/kernel_stats_c3.csv
