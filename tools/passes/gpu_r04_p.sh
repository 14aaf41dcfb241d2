# Round-4 pass p: host-buffer calls launched before their input copies (EGES_GATE): the gate
# tests and the host-buffer / latency / wire tests, then C3 (native caller, bench) and C1 with
# the gate on and off, alternating.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04_p
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_gate.py tests/test_gpu_sender_fused.py tests/test_gpu_raw.py tests/test_c1.py tests/test_gpu_lat.py tests/test_gpu_tri.py tests/test_gpu_exceptional.py tests/test_gpu_handoff.py -x -v --timeout 200 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
bb() {  # name n env...
  local name=$1 n=$2; shift 2
  env "$@" timeout -k 10 120 tools/block_bench $n 300 > $O/bb_${name}.json 2>&1
  python -c "import json; a=json.load(open('$O/bb_${name}.json')); print('bb $name', a['median_ms'], a['p99_ms'], a['errors'])"
}
for i in 1 2 3; do
  bb gate_1000_$i 1000 EGES_GATE=1
  bb nogate_1000_$i 1000 EGES_GATE=0
  bb gate_300_$i 300 EGES_GATE=1
  bb nogate_300_$i 300 EGES_GATE=0
done
for i in 1 2; do
  for g in 1 0; do
    EGES_GATE=$g timeout -k 10 200 python bench.py --config c3 --no-cpu-baseline > $O/c3_g${g}_$i.json 2> $O/c3_g${g}_$i.err
    EGES_GATE=$g timeout -k 10 200 python bench.py --config c1 --no-cpu-baseline > $O/c1_g${g}_$i.json 2> $O/c1_g${g}_$i.err
    python -c "import json; a=json.load(open('$O/c3_g${g}_$i.json')); b=json.load(open('$O/c1_g${g}_$i.json')); print('gate $g c3', a['value'], a['p99_ms'], 'c1', b.get('ms_per_batch'), b.get('p99_ms'))"
  done
done
echo done rc=0
