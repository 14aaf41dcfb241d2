# Round-6 pass o: the 300k lane-serial verify test, now also item for item against the reference.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06_o
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread "tests/test_gpu_workloads.py::test_verify_lane_serial_multi_item" > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -3 $O/pytest.txt
