# C1 (10k transfers from wire bytes): kernel trace + stats of the fused path, the host copy probe,
# and the bucket-form phases of the product build and of diag variants given by suffix.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/c1k_${1:-a}
mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --config c1 --no-cpu-baseline --steps 20 > $O/c1.json 2> $O/c1.err
cat $O/c1.json
find $O/prof -name "*kernel_stats.csv" -exec cat {} \;
timeout -k 10 100 python tools/memcpy_probe.py > $O/memcpy.txt 2>&1
cat $O/memcpy.txt
timeout -k 10 200 python tools/phases_mid.py 10000 > $O/phases.txt 2>&1
cat $O/phases.txt
for v in ${2:-}; do
  EGES_DIAG_LIB=libeges_diag_$v.so timeout -k 10 200 python tools/phases_mid.py 10000 > $O/phases_$v.txt 2>&1
  echo "== variant $v"; cat $O/phases_$v.txt
done
