# Bench alternative builds of libeges.so (eges_amd/libeges_<tag>.so) against the default one.
# Usage (via gpurun): bash tools/variants.sh tag1 tag2 ...
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
cp eges_amd/libeges.so /tmp/libeges_default.so
for tag in default "$@"; do
  if [ "$tag" = default ]; then cp /tmp/libeges_default.so eges_amd/libeges.so; else cp "eges_amd/libeges_$tag.so" eges_amd/libeges.so; fi
  timeout -k 10 120 python bench.py --no-cpu-baseline --steps 10 > "gpurun_out/var_$tag.json" 2> "gpurun_out/var_$tag.err"
  python -c "import json,sys; d=json.load(open('gpurun_out/var_$tag.json')); print('$tag', d['value'], d['roofline']['kernel_ms'], d['config']['correct'])"
done
cp /tmp/libeges_default.so eges_amd/libeges.so
