# Round-4 pass m: a small job's round trip by launch + sync against a resident polling workgroup.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04_m
mkdir -p $O
for i in 1 2; do
  timeout -k 10 60 tools/resident_probe > $O/resident_$i.json 2>&1 || { cat $O/resident_$i.json; exit 1; }
  cat $O/resident_$i.json
done
echo done rc=0
