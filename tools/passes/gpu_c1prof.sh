# C1 (10k transfers from wire bytes) kernel breakdown under rocprofv3, both tx_rows forms, plus
# the form curve at the small end.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/c1prof_${1:-a}
mkdir -p $O
for w in 0 16384; do
  EGES_TXROWS_WAVE_MAX=$w timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_w$w -o run --output-format csv -- python3 bench.py --config c1 --no-cpu-baseline --steps 5 > $O/c1_w$w.json 2> $O/c1_w$w.err
  cat $O/c1_w$w.json
  find $O/prof_w$w -name "*kernel_stats.csv" -exec cat {} \;
done
FORMCURVE_REPS=21 timeout -k 10 300 python tools/formcurve.py 1000,1280,1536,1792,2048,2560,10000 > $O/formcurve_small.jsonl 2> $O/formcurve_small.err
cat $O/formcurve_small.jsonl
