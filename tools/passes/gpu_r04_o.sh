# Round-4 pass o: the resident block server (C3-size blocks): its tests and the latency /
# concurrency tests, then C3 (native caller and bench) with the server on and off, alternating.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04_o
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_resident.py -x -v --timeout 120 --timeout-method thread > $O/pytest_res.txt 2>&1 || { tail -40 $O/pytest_res.txt; exit 1; }
tail -1 $O/pytest_res.txt
EGES_RESIDENT_BLOCK=1 timeout -k 10 500 python -u -m pytest tests/test_gpu_concurrency.py tests/test_gpu_exceptional.py tests/test_gpu_lat.py tests/test_gpu_tri.py tests/test_gpu_sender_fused.py tests/test_c1.py -x -v --timeout 200 --timeout-method thread > $O/pytest_more.txt 2>&1 || { tail -40 $O/pytest_more.txt; exit 1; }
tail -1 $O/pytest_more.txt
bb() {  # name n env...
  local name=$1 n=$2; shift 2
  env "$@" timeout -k 10 120 tools/block_bench $n 300 > $O/bb_${name}.json 2>&1
  python -c "import json; a=json.load(open('$O/bb_${name}.json')); print('bb $name', a['median_ms'], a['p99_ms'], a['errors'])"
}
for i in 1 2 3; do
  bb res_1000_$i 1000 EGES_RESIDENT_BLOCK=1
  bb lane_1000_$i 1000 EGES_RESIDENT_BLOCK=0
  bb res_600_$i 600 EGES_RESIDENT_BLOCK=1
  bb lane_600_$i 600 EGES_RESIDENT_BLOCK=0
done
for i in 1 2; do
  EGES_RESIDENT_BLOCK=1 timeout -k 10 200 python bench.py --config c3 --no-cpu-baseline > $O/c3_res_$i.json 2> $O/c3_res_$i.err
  EGES_RESIDENT_BLOCK=0 timeout -k 10 200 python bench.py --config c3 --no-cpu-baseline > $O/c3_lane_$i.json 2> $O/c3_lane_$i.err
  python -c "import json; a=json.load(open('$O/c3_res_$i.json')); b=json.load(open('$O/c3_lane_$i.json')); print('c3 res', a['value'], a['p99_ms'], 'lane', b['value'], b['p99_ms'])"
done
echo done rc=0
