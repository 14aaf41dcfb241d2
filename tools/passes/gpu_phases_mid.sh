# Mid-size kernel phase stamps (diagnostic builds) at a few batch sizes; extra libs by suffix.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/phases_mid_${1:-a}
mkdir -p $O
timeout -k 10 200 python tools/phases_mid.py ${2:-4096 10000 16384} > $O/phases.txt 2>&1
cat $O/phases.txt
for v in ${3:-}; do
  EGES_DIAG_LIB=libeges_diag_$v.so timeout -k 10 200 python tools/phases_mid.py ${2:-10000} > $O/phases_$v.txt 2>&1
  echo "== variant $v"; cat $O/phases_$v.txt
done
