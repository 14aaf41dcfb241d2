# Round-4 pass t (final sources): the host-buffer / gate / wire / latency tests, then the perf
# evidence (tools/passes/gpu_evidence_r04.sh perf g: bench line, kernel stats, PMC, every config).
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04_t
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_gate.py tests/test_gpu_host_pipe.py tests/test_c1.py tests/test_gpu_raw.py tests/test_gpu_handoff.py tests/test_gpu_mid.py tests/test_gpu_concurrency.py -x -v --timeout 250 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -60 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
bash tools/passes/gpu_evidence_r04.sh perf g
