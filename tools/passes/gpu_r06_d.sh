# Round-6 pass d: round 5's one-launch form rebuilt with discriminating bits (host_one_probe2.py),
# then the new re-read / clamp tests on the product library.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r06_d
mkdir -p $O
EGES_AB_LIB=tools/abhostone/libeges.so timeout -k 10 400 python -u tools/host_one_probe2.py 32 1,33,17,65,97,1 > $O/probe.txt 2>&1 || { tail -20 $O/probe.txt; exit 1; }
cat $O/probe.txt
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_gate.py tests/test_gpu_resident.py tests/test_gpu_host_pipe.py > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -3 $O/pytest.txt
echo done
