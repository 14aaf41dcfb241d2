# Round-4 pass s: the narrow form over width-6 NAF digits (EGES_LAT_WNAF, odd-multiple R' table):
# the latency / exceptional / parity tests, then C3 / single-call / verify A/B against the
# EGES_LAT_WNAF=0 build (tools/abnaf0), alternating.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04_s
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_lat.py tests/test_gpu_exceptional.py tests/test_gpu_parity.py tests/test_gpu_sender_fused.py tests/test_gpu_resident.py tests/test_gpu_concurrency.py tests/test_gpu_handoff.py tests/test_gpu_raw.py -x -v --timeout 250 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -60 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
bb() {  # name n env...
  local name=$1 n=$2; shift 2
  env "$@" timeout -k 10 120 tools/block_bench $n 300 > $O/bb_${name}.json 2>&1
  python -c "import json; a=json.load(open('$O/bb_${name}.json')); print('bb $name', a['median_ms'], a['p99_ms'], a['errors'])"
}
sb() {
  local name=$1; shift
  env "$@" timeout -k 10 120 tools/single_bench 16 2000 > $O/single_${name}.json 2>&1
  python -c "import json; a=json.load(open('$O/single_${name}.json')); print('single $name', a['p50_ms_one_caller'], a['verify_p50_ms_one_caller'], a['recoveries_per_s'], a['errors'])"
}
for i in 1 2 3; do
  bb naf_1000_$i 1000
  bb win_1000_$i 1000 LD_LIBRARY_PATH=$PWD/tools/abnaf0
  bb naf_600_$i 600
  bb win_600_$i 600 LD_LIBRARY_PATH=$PWD/tools/abnaf0
  bb naf_1_$i 1
  bb win_1_$i 1 LD_LIBRARY_PATH=$PWD/tools/abnaf0
done
sb naf
sb win LD_LIBRARY_PATH=$PWD/tools/abnaf0
echo done rc=0
