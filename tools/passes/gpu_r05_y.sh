# Round-5 pass y: the row-form field tests with the worst-magnitude product (FR_MULSUB_MAX), then the
# PMC passes again for the current source hash (selftest.hip is part of it)
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r05_y
timeout -k 10 300 python -u -m pytest tests/test_gpu_fr.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r05_y/pytest_fr.txt 2>&1 || { tail -30 gpurun_out/r05_y/pytest_fr.txt; exit 1; }
tail -1 gpurun_out/r05_y/pytest_fr.txt
bash tools/pmc.sh > gpurun_out/r05_y/pmc.log 2>&1
tail -2 gpurun_out/r05_y/pmc.log
echo done rc=0
