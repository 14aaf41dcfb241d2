# Round-4 pass e: the chunked host-buffer path by chunk count (EGES_HOST_PARTS, reused output
# arrays), then the default bench line (C2 + secondary, c2_host included).
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04_e
mkdir -p $O
c2h() {  # name env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --config c2host --steps 8 --warmup 2 > $O/c2host_$name.json 2> $O/c2host_$name.err
  python -c "import json; a=json.load(open('$O/c2host_$name.json')); print('c2host $name', a['value'], a['ms_per_step'], a['fresh_outputs_sigs_per_s'], a['config']['correct'])"
}
for i in 1 2; do
  for p in 2 3 4 5 6 8; do
    c2h parts${p}_$i EGES_HOST_PIPE=0 EGES_HOST_PARTS=$p
  done
done
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
python - <<'PY'
import json
d = json.load(open("gpurun_out/r04_e/bench.json"))
print("c2", d["value"], d["roofline"]["kernel_ms"], d["config"]["correct"])
for k, v in d["secondary"].items():
    if isinstance(v, dict):
        print(k, {a: b for a, b in v.items() if a not in ("roofline", "kinds", "path", "cpu")}, (v.get("roofline") or {}).get("kernel_ms"))
PY
echo done rc=0
