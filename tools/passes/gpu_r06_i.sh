# Round-6 pass i: the resident tests and the default bench line (new counters / baseline / tax fields).
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r06_i
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_resident.py tests/test_capi.py > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
grep "other process" $O/pytest.txt || true
tail -1 $O/pytest.txt
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
python -c "
import json; a=json.load(open('$O/bench.json'))
print(a['value'], a['config']['correct'])
print(json.dumps(a['cpu_baseline'])[:900])
print(json.dumps(a['secondary']['single']))
"
echo done
