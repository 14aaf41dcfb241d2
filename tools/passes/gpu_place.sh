# Latency-kernel placement probe: which SIMD each signature's waves run on (stamped build,
# hw_place) and the Strauss ticks by SIMD sharing, at the C3 size and at sizes where every
# signature has its SIMDs alone.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/place_${1:-a}
mkdir -p $O
for n in ${2:-1000 256 512 2000}; do
  EGES_LAT_WIDE_MAX=0 timeout -k 10 120 python tools/phases.py $n > $O/phases_n$n.txt 2>&1 || { cat $O/phases_n$n.txt; exit 1; }
  cat $O/phases_n$n.txt
done
