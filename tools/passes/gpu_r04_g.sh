# Round-4 pass g: the latency kernel's three-wave form: its tests, then C3 (native caller) against
# the narrow form, alternating, and the split point (EGES_TRI_W0 17 / 20 / 23 builds).
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04_g
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_tri.py tests/test_gpu_exceptional.py tests/test_gpu_lat.py tests/test_gpu_handoff.py -x -v --timeout 200 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
bb() {  # name n env...
  local name=$1 n=$2; shift 2
  env "$@" timeout -k 10 120 tools/block_bench $n 300 > $O/bb_${name}.json 2>&1
  python -c "import json; a=json.load(open('$O/bb_${name}.json')); print('bb $name', a['median_ms'], a['p99_ms'], a['errors'])"
}
for i in 1 2 3; do
  bb narrow_1000_$i 1000 EGES_LAT_TRI_MAX=0
  bb tri_1000_$i 1000 EGES_LAT_TRI_MAX=1536
  bb tri17_1000_$i 1000 EGES_LAT_TRI_MAX=1536 LD_LIBRARY_PATH=$PWD/tools/abtri17
  bb tri23_1000_$i 1000 EGES_LAT_TRI_MAX=1536 LD_LIBRARY_PATH=$PWD/tools/abtri23
done
for n in 300 600 800; do
  bb narrow_$n $n EGES_LAT_TRI_MAX=0
  bb tri_$n $n EGES_LAT_TRI_MAX=1536
done
echo done rc=0
