# Round-5 pass b: the reference-pinned workload tests (C3 block, 1M VerifySignature mix), then the
# default bench line's multi-rank path rehearsed with 2 ranks on the one GPU (gloo): the c4_strong
# leg and rank 0's c4host child over 2 logical devices.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r05_b
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_workloads.py -x -v --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
export EGES_BENCH_DEVICE=0 EGES_BENCH_BACKEND=gloo EGES_TEST_LOGICAL_DEVICES=2
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 > $O/dist2_c2.json 2> $O/dist2_c2.err || { tail -30 $O/dist2_c2.err; exit 1; }
cat $O/dist2_c2.json
echo done rc=0
