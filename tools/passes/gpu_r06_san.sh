# Round-6: the host-code ASan/UBSan harness on the GPU (tools/sanitize_host.cpp, libeges_asan.so)
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/ev6_a
mkdir -p $O
ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1 timeout -k 10 300 tools/asan/sanitize_host 5000 > $O/sanitize_gpu.log 2>&1 || { tail -30 $O/sanitize_gpu.log; exit 1; }
tail -3 $O/sanitize_gpu.log
