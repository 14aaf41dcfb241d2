# Split (4-wave) vs narrow (2-wave + root helpers) launch time by batch size, alternating.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for n in 64 128 192 256 384; do
  for w in 0 100000; do
    EGES_LAT_WIDE_MAX=$w timeout -k 10 100 python tools/phases.py $n > gpurun_out/xo_${n}_$w.txt 2>&1
    echo "n=$n wide_max=$w $(grep launch gpurun_out/xo_${n}_$w.txt) $(grep per-wave gpurun_out/xo_${n}_$w.txt)"
  done
done
