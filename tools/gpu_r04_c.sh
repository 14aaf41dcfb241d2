# Round-4 pass c: scalar-ALU divsteps in assembly. Row-form field/inverse tests, the inversion
# latency A/B (asm vs compiled C, same box, alternating), latency-kernel and exceptional tests,
# then C3 native block call and single-call latency A/B (tools/abbase = the C divsteps build).
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04_c
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_fr.py -x -v -s --timeout 200 --timeout-method thread > $O/pytest_fr.txt 2>&1 || { tail -30 $O/pytest_fr.txt; exit 1; }
grep -E "inversion|passed|failed" $O/pytest_fr.txt
timeout -k 10 120 python tools/ab_inv.py 3 > $O/ab_inv.json 2>&1
cat $O/ab_inv.json
timeout -k 10 600 python -u -m pytest tests/test_gpu_lat.py tests/test_gpu_exceptional.py tests/test_gpu_parity.py tests/test_gpu_concurrency.py -x -v --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for i in 1 2 3; do
  timeout -k 10 120 tools/block_bench 1000 300 > $O/bb_asm_$i.json 2>&1
  LD_LIBRARY_PATH=$PWD/tools/abbase timeout -k 10 120 tools/block_bench 1000 300 > $O/bb_c_$i.json 2>&1
  cat $O/bb_asm_$i.json $O/bb_c_$i.json
done
for i in 1 2; do
  timeout -k 10 120 tools/single_bench 1 300 > $O/single_asm_$i.json 2>&1
  LD_LIBRARY_PATH=$PWD/tools/abbase timeout -k 10 120 tools/single_bench 1 300 > $O/single_c_$i.json 2>&1
  cat $O/single_asm_$i.json $O/single_c_$i.json
done
timeout -k 10 120 tools/memcpy_probe > $O/memcpy_probe.txt 2>&1
cat $O/memcpy_probe.txt
timeout -k 10 200 python bench.py --config c2host --steps 5 --warmup 2 > $O/c2host.json 2> $O/c2host.err
cat $O/c2host.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c2host -o run --output-format csv -- python3 bench.py --config c2host --steps 3 --warmup 1 > $O/prof_c2host.log 2>&1
for b in 65536 131072 262144 524288 1048576; do
  timeout -k 10 120 python bench.py --batch $b --steps 5 --warmup 2 --no-secondary --no-cpu-baseline > $O/c2_b$b.json 2> $O/c2_b$b.err
  python -c "import json,sys; d=json.load(open('$O/c2_b$b.json')); print($b, d['roofline']['kernel_ms'], d['value'])"
done
