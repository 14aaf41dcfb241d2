# Round-6 pass q: does the host's wait for the stream cost C3 / C1 time? The same build with the
# runtime's active-wait window at its default and raised (ROC_ACTIVE_WAIT_TIMEOUT, us), alternating.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06_q
mkdir -p $O
for i in 1 2 3; do
  for v in def spin; do
    E=; [ $v = spin ] && E="ROC_ACTIVE_WAIT_TIMEOUT=100000"
    env $E timeout -k 10 200 python bench.py --config c3 --no-cpu-baseline > $O/c3_${v}_$i.json 2> $O/c3_${v}_$i.err
    env $E timeout -k 10 200 python bench.py --config c1 --no-cpu-baseline > $O/c1_${v}_$i.json 2> $O/c1_${v}_$i.err
    env $E timeout -k 10 120 tools/block_bench 1000 300 > $O/block_${v}_$i.json 2>&1
    python -c "
import json; a=json.load(open('$O/c3_${v}_$i.json')); b=json.load(open('$O/c1_${v}_$i.json')); c=json.load(open('$O/block_${v}_$i.json'))
print('$v', 'c3', a['value'], a['roofline']['kernel_ms'], 'c1', b.get('ms_per_batch'), 'block native', c['median_ms'])"
  done
done
echo done
