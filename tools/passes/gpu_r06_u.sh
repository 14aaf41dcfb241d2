# Round-6 pass u (probe): is wave 1's signing hash on C3-from-wire's critical path? The product
# build against a probe build whose wave 1 skips the hash (wrong addresses on purpose: timing only).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06_u
mkdir -p $O
for i in 1 2 3; do
  for v in prod nohash; do
    L=; [ $v = nohash ] && L=tools/abnohash/libeges.so
    EGES_AB_LIB=$L timeout -k 10 200 python bench.py --config c3raw --no-cpu-baseline > $O/c3raw_${v}_$i.json 2> $O/c3raw_${v}_$i.err
    rc=$?
    [ $rc -gt 1 ] && { echo "rc $rc"; tail -5 $O/c3raw_${v}_$i.err; exit 1; }
    python -c "
import json; r=json.load(open('$O/c3raw_${v}_$i.json'))
print('$v', r['value'], r['roofline']['kernel_ms'], r['config']['correct'])"
  done
done
echo done
