# C2 A/B on one box, alternating: a single-chunk 1M batch as one launch (default) vs two
# launches overlapped on two streams (EGES_OVERLAP=2). bench.py times the
# step span with HIP events on the engine's stream either way.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/c2ov_${1:-a}
mkdir -p $O
for rep in 1 2 3; do
  for v in base ov2; do
    if [ $v = ov2 ]; then export EGES_OVERLAP=2; else unset EGES_OVERLAP; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary --steps 20 > $O/c2_${v}_$rep.json 2> $O/c2_${v}_$rep.err
    python -c "import json,sys; d=json.load(open('$O/c2_${v}_$rep.json')); print('$v', $rep, d['value'], d['roofline']['kernel_ms'], d['config']['correct'])"
  done
done
