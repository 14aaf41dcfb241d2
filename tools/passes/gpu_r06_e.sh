# Round-6 pass e: (1) more statistics on the rebuilt one-launch form, alternating mode 1 (no
# read-back) and 65 (system-scope read-back before each block's done word); (2) the GPU tests of the
# publication paths on the product library with the read-back in gate_done and the resident
# server; (3) C1 and single-call timing with the read-back (bench.py --config c1, single_bench).
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r06_e
mkdir -p $O
EGES_AB_LIB=tools/abhostone/libeges.so timeout -k 10 500 python -u tools/host_one_probe2.py 48 1,65,1,65 > $O/probe.txt 2>&1 || { tail -20 $O/probe.txt; exit 1; }
cat $O/probe.txt | cut -c1-300
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_gate.py tests/test_gpu_resident.py tests/test_gpu_mid.py tests/test_gpu_handoff.py > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
for i in 1 2; do
timeout -k 10 200 python bench.py --config c1 > $O/bench_c1_$i.json 2> $O/bench_c1_$i.err
python -c "import json; a=json.load(open('$O/bench_c1_$i.json')); print('c1', a['value'], a['ms_per_step'], a.get('config',{}).get('correct'))"
timeout -k 10 200 tools/single_bench 1 3000 > $O/single1_$i.json 2> $O/single1_$i.err
cat $O/single1_$i.json | cut -c1-300
done
echo done
