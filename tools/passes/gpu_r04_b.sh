# Round-4 pass b: every GPU test (fused sender rows, hand-offs, asm divsteps, host pipeline, the
# 1M reference checks), then same-box A/Bs: inversion latency (asm vs C divsteps), the C3 native
# block call (asm vs C lib; fused sender rows on / off), single-call latency, the host-buffer
# pipeline (on / off, chunk schedules), copy rates, and the lane-serial kernel vs batch size.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04_b
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { tail -40 $O/pytest_gpu.txt; exit 1; }
tail -1 $O/pytest_gpu.txt
grep -E "inversion|squaring" $O/pytest_gpu.txt || true
timeout -k 10 120 python tools/ab_inv.py 3 > $O/ab_inv.json 2>&1
cat $O/ab_inv.json
for i in 1 2 3; do
  timeout -k 10 120 tools/block_bench 1000 300 > $O/bb_asm_$i.json 2>&1
  LD_LIBRARY_PATH=$PWD/tools/abbase timeout -k 10 120 tools/block_bench 1000 300 > $O/bb_c_$i.json 2>&1
  EGES_SENDER_FUSED=0 timeout -k 10 120 tools/block_bench 1000 300 > $O/bb_nofuse_$i.json 2>&1
  cat $O/bb_asm_$i.json $O/bb_c_$i.json $O/bb_nofuse_$i.json
done
timeout -k 10 120 tools/block_bench_diag 1000 300 > $O/bb_diag.json 2>&1 && cat $O/bb_diag.json
timeout -k 10 120 tools/block_bench_diag 1 300 > $O/bb_diag_n1.json 2>&1 && cat $O/bb_diag_n1.json
for i in 1 2; do
  timeout -k 10 120 tools/single_bench 16 2000 > $O/single_asm_$i.json 2>&1
  LD_LIBRARY_PATH=$PWD/tools/abbase timeout -k 10 120 tools/single_bench 16 2000 > $O/single_c_$i.json 2>&1
  cat $O/single_asm_$i.json $O/single_c_$i.json
done
timeout -k 10 120 tools/memcpy_probe > $O/memcpy_probe.txt 2>&1
cat $O/memcpy_probe.txt
for i in 1 2; do
  timeout -k 10 200 python bench.py --config c2host --steps 5 --warmup 2 > $O/c2host_pipe_$i.json 2> $O/c2host_pipe_$i.err
  EGES_HOST_PIPE=0 timeout -k 10 200 python bench.py --config c2host --steps 5 --warmup 2 > $O/c2host_old_$i.json 2> $O/c2host_old_$i.err
  python -c "import json; a=json.load(open('$O/c2host_pipe_$i.json')); b=json.load(open('$O/c2host_old_$i.json')); print('c2host pipe', a['value'], a['config']['correct'], 'old', b['value'], b['config']['correct'])"
done
for fc in 65536:262144 131072:349526 262144:262144 131072:524288; do
  f=${fc%%:*}; c=${fc##*:}
  EGES_PIPE_FIRST=$f EGES_PIPE_CHUNK=$c timeout -k 10 200 python bench.py --config c2host --steps 5 --warmup 2 > $O/c2host_${f}_$c.json 2> $O/c2host_${f}_$c.err
  python -c "import json; a=json.load(open('$O/c2host_${f}_$c.json')); print('c2host first $f chunk $c', a['value'], a['config']['correct'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c2host -o run --output-format csv -- python3 bench.py --config c2host --steps 3 --warmup 1 > $O/prof_c2host.log 2>&1
for b in 65536 131072 262144 524288 1048576; do
  timeout -k 10 120 python bench.py --batch $b --steps 5 --warmup 2 --no-secondary --no-cpu-baseline > $O/c2_b$b.json 2> $O/c2_b$b.err
  python -c "import json; d=json.load(open('$O/c2_b$b.json')); print('lane-serial batch', $b, 'kernel_ms', d['roofline']['kernel_ms'], 'sigs/s', d['value'])"
done
timeout -k 10 300 python tools/formcurve_verify.py > $O/formcurve_verify.jsonl 2> $O/formcurve_verify.err
tail -1 $O/formcurve_verify.jsonl
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --config c1 --steps 5 --no-cpu-baseline > $O/c1_binv_$i.json 2> $O/c1_binv_$i.err
  EGES_AB_LIB=$PWD/tools/abmid/libeges.so timeout -k 10 200 python bench.py --config c1 --steps 5 --no-cpu-baseline > $O/c1_lane_$i.json 2> $O/c1_lane_$i.err
  python -c "import json; a=json.load(open('$O/c1_binv_$i.json')); b=json.load(open('$O/c1_lane_$i.json')); print('c1 batchinv', a['ms_per_batch'], a['roofline']['kernel_ms'], 'per-lane inv', b['ms_per_batch'], b['roofline']['kernel_ms'], a['config']['correct'], b['config']['correct'])"
done
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 10 --no-secondary --no-cpu-baseline > $O/c2_binv_$i.json 2> $O/c2_binv_$i.err
  EGES_AB_LIB=$PWD/tools/abmid/libeges.so timeout -k 10 200 python bench.py --steps 10 --no-secondary --no-cpu-baseline > $O/c2_lane_$i.json 2> $O/c2_lane_$i.err
  python -c "import json; a=json.load(open('$O/c2_binv_$i.json')); b=json.load(open('$O/c2_lane_$i.json')); print('c2 wave-batch inv', a['value'], a['roofline']['kernel_ms'], 'per-thread inv', b['value'], b['roofline']['kernel_ms'], a['config']['correct'], b['config']['correct'])"
done
