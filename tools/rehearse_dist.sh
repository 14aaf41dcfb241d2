# Rehearse bench.py's multi-process path on a 1-GPU box: 2 ranks launched by torch.distributed.run
# exactly as the driver does, both on cuda:0, gloo for the barrier / max-over-ranks collectives.
set -e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
export EGES_BENCH_DEVICE=0 EGES_BENCH_BACKEND=gloo
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 > gpurun_out/dist2_c2.json 2> gpurun_out/dist2_c2.err
cat gpurun_out/dist2_c2.json
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29534 bench.py --gpus 2 --steps 2 --warmup 1 --config c4 --batch 8388608 > gpurun_out/dist2_c4.json 2> gpurun_out/dist2_c4.err
cat gpurun_out/dist2_c4.json
