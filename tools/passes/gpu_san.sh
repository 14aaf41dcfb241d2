# The host-code harness on the GPU: the plain build (product libeges.so) first, then the
# ASan/UBSan build; kernel-level logging on the ASan run to name a faulting dispatch.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/san_${1:-a}
mkdir -p $O
timeout -k 10 300 tools/sanitize_host_plain 2000 > $O/plain.log 2>&1
echo "plain rc=$?"; grep -v "^MISMATCH.*mutation" $O/plain.log | tail -5
AMD_LOG_LEVEL=1 ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 timeout -k 10 300 tools/asan/sanitize_host 2000 > $O/asan.log 2>&1
echo "asan rc=$?"; grep -v "^MISMATCH.*mutation" $O/asan.log | tail -20
