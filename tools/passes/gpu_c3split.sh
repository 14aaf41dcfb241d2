# C3 block bench with the narrow (2-wave) vs split (4-wave) latency form, alternating.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for rep in 1 2; do
  for w in 256 2000; do
    EGES_LAT_WIDE_MAX=$w timeout -k 10 200 python bench.py --config c3 --no-cpu-baseline > gpurun_out/c3w_${w}_$rep.json 2> gpurun_out/c3w.err
    python -c "import json;b=json.load(open('gpurun_out/c3w_${w}_$rep.json'));print('wide_max=$w rep=$rep', b['value'], b['p99_ms'], b['config']['correct'])"
  done
done
