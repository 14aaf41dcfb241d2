# Round-6 pass t: the root helpers touch every line of a wire-format item before decoding it (one
# bus round trip instead of one per RLP head). Tests of the wire paths, then same-box A/B against
# the previous build (tools/abpf): C3 from wire bytes, C3, C1 (bench.py configs), alternating.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06_t
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_raw.py tests/test_gpu_rlp.py tests/test_c1.py tests/test_gpu_lat.py tests/test_gpu_tri.py > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for i in 1 2 3; do
  for v in new old; do
    L=; [ $v = old ] && L=tools/abpf/libeges.so
    for c in c3raw c3 c1; do
      EGES_AB_LIB=$L timeout -k 10 200 python bench.py --config $c --no-cpu-baseline > $O/${c}_${v}_$i.json 2> $O/${c}_${v}_$i.err
    done
    python -c "
import json
r=[json.load(open('$O/%s_${v}_$i.json' % c)) for c in ('c3raw','c3','c1')]
print('$v', 'c3raw', r[0]['value'], r[0]['roofline']['kernel_ms'], 'c3', r[1]['value'], r[1]['roofline']['kernel_ms'], 'c1', r[2].get('ms_per_batch'), all(x['config']['correct'] for x in r))"
  done
done
echo done
