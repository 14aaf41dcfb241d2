# Round-6 pass c: round 5's one-launch host form rebuilt with discriminating bits
# (tools/abhostone/libeges.so from f000a43 + probe bits; tools/host_one_probe2.py).
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r06_c
mkdir -p $O
EGES_AB_LIB=tools/abhostone/libeges.so timeout -k 10 400 python -u tools/host_one_probe2.py 32 1,33,17,65,97,1 > $O/probe.txt 2>&1 || { tail -20 $O/probe.txt; exit 1; }
cat $O/probe.txt
echo done
