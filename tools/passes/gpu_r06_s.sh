# Round-6 pass s: the routing-cut test.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06_s
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_routing.py > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -4 $O/pytest.txt
