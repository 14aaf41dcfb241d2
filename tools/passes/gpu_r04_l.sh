# Round-4 pass l: HIP runtime settings that touch a small call's launch and completion latency
# (kernel arguments in device memory, the host's active-wait window), on C3 and single calls;
# the split form's join order (R sums on E' first) against the previous build; phase stamps.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04_l
mkdir -p $O
bb() {  # name n env...
  local name=$1 n=$2; shift 2
  env "$@" timeout -k 10 120 tools/block_bench $n 300 > $O/bb_${name}.json 2>&1
  python -c "import json; a=json.load(open('$O/bb_${name}.json')); print('bb $name', a['median_ms'], a['p99_ms'], a['errors'])"
}
sb() {
  local name=$1; shift
  env "$@" timeout -k 10 120 tools/single_bench 16 2000 > $O/single_${name}.json 2>&1
  python -c "import json; a=json.load(open('$O/single_${name}.json')); print('single $name', a['p50_ms_one_caller'], a['verify_p50_ms_one_caller'], a['recoveries_per_s'], a['errors'])"
}
for i in 1 2; do
  bb def_1000_$i 1000
  bb devka_1000_$i 1000 HIP_FORCE_DEV_KERNARG=1
  bb def_1_$i 1
  bb devka_1_$i 1 HIP_FORCE_DEV_KERNARG=1
  bb wait_1_$i 1 ROC_ACTIVE_WAIT_TIMEOUT=1000
  sb def_$i
  sb devka_$i HIP_FORCE_DEV_KERNARG=1
done
for i in 1 2 3; do
  bb ord_new_1_$i 1
  bb ord_old_1_$i 1 LD_LIBRARY_PATH=$PWD/tools/abprev
  bb ord_new_200_$i 200
  bb ord_old_200_$i 200 LD_LIBRARY_PATH=$PWD/tools/abprev
  sb ord_new_$i
  sb ord_old_$i LD_LIBRARY_PATH=$PWD/tools/abprev
done
for n in 1 16 1000; do
  timeout -k 10 120 python tools/phases.py $n > $O/phases_n$n.txt 2>&1 || { tail -20 $O/phases_n$n.txt; exit 1; }
done
head -14 $O/phases_n1.txt
echo done rc=0
