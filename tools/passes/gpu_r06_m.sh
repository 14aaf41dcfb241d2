# Round-6 pass m: the DPP-layout wave Keccak: the tests of every path that uses it (latency forms'
# addresses, wire-format signing hashes), then same-box A/B against the previous build
# (tools/abkec): C3 (bench, native), C3 from wire bytes, single recover p50.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r06_m
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_lat.py tests/test_gpu_raw.py tests/test_gpu_parity.py tests/test_gpu_tri.py tests/test_gpu_block.py tests/test_gpu_rlp.py tests/test_c1.py tests/test_gpu_resident.py > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for i in 1 2 3; do
  for v in new old; do
    L=; S=tools/single_bench; B=tools/block_bench
    [ $v = old ] && L=tools/abkec/libeges.so && S=tools/abkec/single_bench && B=tools/abkec/block_bench
    EGES_AB_LIB=$L timeout -k 10 200 python bench.py --config c3 --no-cpu-baseline > $O/c3_${v}_$i.json 2> $O/c3_${v}_$i.err
    EGES_AB_LIB=$L timeout -k 10 200 python bench.py --config c3raw --no-cpu-baseline > $O/c3raw_${v}_$i.json 2> $O/c3raw_${v}_$i.err
    python -c "
import json; a=json.load(open('$O/c3_${v}_$i.json')); b=json.load(open('$O/c3raw_${v}_$i.json'))
print('c3 $v', a['value'], a['roofline']['kernel_ms'], a['config']['correct'], 'c3raw', b['value'], b['roofline']['kernel_ms'], b['config']['correct'])"
    timeout -k 10 200 $S 1 3000 > $O/single_${v}_$i.json 2> $O/single_${v}_$i.err
    timeout -k 10 200 $B 1000 300 > $O/block_${v}_$i.json 2>&1
    python -c "
import json; a=json.load(open('$O/single_${v}_$i.json')); b=json.load(open('$O/block_${v}_$i.json'))
print('single $v', a['p50_ms_one_caller'], a['verify_p50_ms_one_caller'], 'block native', b['median_ms'])"
  done
done
echo done
