# Round-5 pass f: which side a stale byte of the one-launch host form comes from (tools/host_one_probe.py),
# then the host-pipe tests and the c2host A/B.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r05_f
mkdir -p $O
timeout -k 10 300 python -u tools/host_one_probe.py 16 1,3,5,7,0,8,9,10 > $O/probe.txt 2>&1 || { tail -20 $O/probe.txt; exit 1; }
cat $O/probe.txt
for i in 1 2; do
  for v in 1_4_0 1_4_6 1_1_0 0_4_0; do
    IFS=_ read one fd tm <<< "$v"
    EGES_HOST_ONE=$one EGES_HOST_FEEDERS=$fd EGES_TEST_HOST_ONE=$tm timeout -k 10 120 python bench.py --config c2host --steps 8 --warmup 2 > $O/c2host_${v}_$i.json 2> $O/c2host_${v}_$i.err
    python -c "import json; a=json.load(open('$O/c2host_${v}_$i.json')); print('c2host one_feeders_mode=$v', a['value'], a['ms_per_step'], a['fresh_outputs_sigs_per_s'], a['config']['correct'])"
  done
done
EGES_HOST_ONE=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_one -o run --output-format csv -- python bench.py --config c2host --steps 6 --warmup 1 > $O/prof_one.log 2>&1
EGES_HOST_ONE=1 EGES_TEST_HOST_ONE=8 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_pre -o run --output-format csv -- python bench.py --config c2host --steps 6 --warmup 1 > $O/prof_pre.log 2>&1
find $O/prof_one $O/prof_pre -name "*kernel_stats*" | while read f; do echo $f; head -4 $f; done
echo done rc=0
