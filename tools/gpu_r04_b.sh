# Round-4 pass b: fused sender rows (no prep_sender launch) — GPU tests of the sender paths, then
# a same-box A/B of the C3 native block call (EGES_SENDER_FUSED 1 vs 0, alternating).
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04_b
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_sender_fused.py tests/test_gpu_parity.py tests/test_gpu_types_host.py tests/test_gpu_mid.py tests/test_gpu_lat.py tests/test_gpu_handoff.py -x -v --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for i in 1 2 3; do
  EGES_SENDER_FUSED=1 timeout -k 10 120 tools/block_bench_diag 1000 300 > $O/bb_f1_$i.json 2>&1
  EGES_SENDER_FUSED=0 timeout -k 10 120 tools/block_bench_diag 1000 300 > $O/bb_f0_$i.json 2>&1
  cat $O/bb_f1_$i.json $O/bb_f0_$i.json
done
