# Round-5 pass zf: the split form's high-window width (EGES_HBITS 4 = default, 3, 5: the high windows and their table of D) after the
# faster row product, same box, alternating: single recover / verify p50 (resident server) and
# a 200-signature batch (split form) through the device entry
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r05_zf
mkdir -p $O
for i in 1 2 3; do
  for v in :tools hb3:tools/abhb3/bin hb5:tools/abhb5/bin; do
    tag=${v%%:*}; b=${v#*:}
    timeout -k 10 120 $b/single_bench 1 3000 > $O/s1_${tag:-hb4}_$i.json 2>&1
    timeout -k 10 120 $b/block_bench 200 300 > $O/bb200_${tag:-hb4}_$i.json 2>&1
    python - $O ${tag:-hb4} $i <<'PY'
import json, sys
o, t, i = sys.argv[1:]
last = lambda f: json.loads(open(f).read().strip().splitlines()[-1])
s1, bb = last(f"{o}/s1_{t}_{i}.json"), last(f"{o}/bb200_{t}_{i}.json")
print(t, i, "single", s1["p50_ms_one_caller"], s1["verify_p50_ms_one_caller"], s1["errors"], "block200", bb["median_ms"], bb["errors"])
PY
  done
done
echo done rc=0
