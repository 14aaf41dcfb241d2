# Wire fusion in the latency kernels (k_recover_lat.hip): the wire-path parity tests on all three
# forms (tx_rows, fused bucket, fused latency), the latency-kernel suites, then C3raw A/B
# (EGES_WIRE_FUSED 1 = latency kernels decode the bytes, 2 = bucket only, so C3raw goes through
# tx_rows_wave + prep_sender), alternating on the same box.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/latwire_${1:-a}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_raw.py tests/test_gpu_rlp.py tests/test_gpu_block.py tests/test_c1.py tests/test_gpu_lat.py tests/test_gpu_parity.py tests/test_gpu_exceptional.py -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for i in 1 2 3; do
  for f in 1 2; do
    EGES_WIRE_FUSED=$f timeout -k 10 200 python bench.py --config c3raw --no-cpu-baseline > $O/c3raw_f${f}_$i.json 2> $O/c3raw_f${f}_$i.err
    echo "fused=$f run $i: $(python -c "import json,sys;d=json.load(open('$O/c3raw_f${f}_$i.json'));print(d['ms_per_step'], d['value'])")"
  done
done
