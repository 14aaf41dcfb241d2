# Round-6 pass f: same-box A/B of the system-scope read-back before the completion words (the
# product library against tools/abprev = commit 3d4ec21 without it): C1 whole call and single
# recover p50, three alternating pairs.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r06_f
mkdir -p $O
for i in 1 2 3; do
  for v in new prev; do
    if [ $v = prev ]; then L=tools/abprev/libeges.so; S=tools/abprev/single_bench; else L=; S=tools/single_bench; fi
    EGES_AB_LIB=$L timeout -k 10 200 python bench.py --config c1 --steps 40 > $O/c1_${v}_$i.json 2> $O/c1_${v}_$i.err
    python -c "import json; a=json.load(open('$O/c1_${v}_$i.json')); print('c1 $v', a['value'], a['ms_per_batch'], a['p99_ms'], a['config']['correct'])"
    timeout -k 10 200 $S 1 3000 > $O/single_${v}_$i.json 2> $O/single_${v}_$i.err
    python -c "import json; a=json.load(open('$O/single_${v}_$i.json')); print('single $v', {k: a[k] for k in a if 'p50' in k or 'p99' in k})"
  done
done
echo done
