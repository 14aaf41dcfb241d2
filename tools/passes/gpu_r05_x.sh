# Round-5 pass x: SIMD placement of a 5-wave workgroup (tools/place_probe.hip)
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r05_x
timeout -k 10 60 tools/place_probe | tee gpurun_out/r05_x/place.txt
echo done rc=0
