# Round-5 pass c: the default bench line's multi-rank path rehearsed with 2 ranks on the one GPU
# (gloo): the c4_strong leg and rank 0's c4host child over 2 logical devices.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r05_c
mkdir -p $O
export EGES_BENCH_DEVICE=0 EGES_BENCH_BACKEND=gloo EGES_TEST_LOGICAL_DEVICES=2
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 > $O/dist2_c2.json 2> $O/dist2_c2.err || { tail -30 $O/dist2_c2.err; exit 1; }
tail -c 2500 $O/dist2_c2.json
echo done rc=0
