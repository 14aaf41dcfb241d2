# Same-box A/B of two library builds (EGES_LIB=libeges_base.so vs libeges.so), alternating:
# bench configs given as $2 (default "c3 c1"), three rounds.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/ab_${1:-a}
mkdir -p $O
for i in 1 2 3; do
  for cfg in ${2:-c3 c1}; do
    for lib in libeges_base.so libeges.so; do
      EGES_LIB=$lib timeout -k 10 200 python bench.py --config $cfg --no-cpu-baseline > $O/${cfg}_${lib%.so}_$i.json 2> $O/${cfg}_${lib%.so}_$i.err
      echo "$cfg $lib run $i: $(python -c "import json;d=json.load(open('$O/${cfg}_${lib%.so}_$i.json'));print(d['value'], d['unit'], d.get('p99_ms'))")"
    done
  done
done
