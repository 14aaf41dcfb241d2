# Round-5 pass w: host-buffer 1M ecrecover from pageable against pinned caller arrays (tools/pinned_probe.py)
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r05_w
timeout -k 10 300 python -u tools/pinned_probe.py 1048576 6 | tee gpurun_out/r05_w/pinned_probe.jsonl
echo done rc=0
