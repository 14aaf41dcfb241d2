# Round-4 pass n: the resident single-call server: its tests and the single-call paths' tests,
# then single calls and small blocks with the server on and off, alternating.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04_n
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_resident.py -x -v --timeout 120 --timeout-method thread > $O/pytest_res.txt 2>&1 || { tail -40 $O/pytest_res.txt; exit 1; }
tail -1 $O/pytest_res.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_concurrency.py tests/test_gpu_exceptional.py tests/test_gpu_lat.py tests/test_gpu_handoff.py -x -v --timeout 200 --timeout-method thread > $O/pytest_more.txt 2>&1 || { tail -40 $O/pytest_more.txt; exit 1; }
tail -1 $O/pytest_more.txt
sb() {
  local name=$1 t=$2; shift 2
  env "$@" timeout -k 10 120 tools/single_bench $t 2000 > $O/single_${name}.json 2>&1
  python -c "import json; a=json.load(open('$O/single_${name}.json')); print('single $name', a['p50_ms_one_caller'], a['p99_ms_one_caller'], a['verify_p50_ms_one_caller'], a['recoveries_per_s'], a['errors'])"
}
for i in 1 2 3; do
  sb res16_$i 16 EGES_RESIDENT=1
  sb lane16_$i 16 EGES_RESIDENT=0
  sb res8_$i 8 EGES_RESIDENT=1
  sb lane8_$i 8 EGES_RESIDENT=0
done
echo done rc=0
