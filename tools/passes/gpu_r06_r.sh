# Round-6 pass r: the concurrency tests, including the new mid-size band one.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06_r
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_concurrency.py > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -8 $O/pytest.txt
