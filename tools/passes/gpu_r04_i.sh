# Round-4 pass i: paired doublings in the latency kernels (frg.cuh gejq_double2): the latency,
# exceptional, three-wave, hand-off and verify tests, then C3 / single / small-n A/B against the
# EGES_LAT_DBL2=0 build, alternating.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04_i
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_lat.py tests/test_gpu_exceptional.py tests/test_gpu_tri.py tests/test_gpu_handoff.py tests/test_gpu_sender_fused.py tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
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
  bb dbl2_1000_$i 1000
  bb dbl1_1000_$i 1000 LD_LIBRARY_PATH=$PWD/tools/abdbl
  bb dbl2_1_$i 1
  bb dbl1_1_$i 1 LD_LIBRARY_PATH=$PWD/tools/abdbl
  sb dbl2_$i
  sb dbl1_$i LD_LIBRARY_PATH=$PWD/tools/abdbl
done
for n in 300 448; do
  bb dbl2_$n $n
  bb dbl1_$n $n LD_LIBRARY_PATH=$PWD/tools/abdbl
done
echo done rc=0
