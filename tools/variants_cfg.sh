# Same-box A/B of alternative builds (eges_amd/libeges_<tag>.so) on one bench config.
# Usage (via gpurun): CFG=c2host bash tools/variants_cfg.sh tag1 tag2 ...
set -e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
CFG=${CFG:-c2}
cp eges_amd/libeges.so /tmp/libeges_default.so
for tag in default "$@" default "$@"; do
  if [ "$tag" = default ]; then cp /tmp/libeges_default.so eges_amd/libeges.so; else cp "eges_amd/libeges_$tag.so" eges_amd/libeges.so; fi
  timeout -k 10 120 python bench.py --config $CFG --no-cpu-baseline --steps 5 > "gpurun_out/var_$tag.json" 2> "gpurun_out/var_$tag.err"
  python -c "import json; d=json.load(open('gpurun_out/var_$tag.json')); print('$tag', d['value'], d['unit'], d['config']['correct'])"
done
cp /tmp/libeges_default.so eges_amd/libeges.so
