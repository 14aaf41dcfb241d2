# Round-3 GPU pass: parity tests, the default bench line (c2 + secondary), optional extra configs.
# Usage (via gpurun, from the repo root): bash tools/passes/gpu_r03.sh TAG [extra bench configs...]
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-a}
shift || true
O=gpurun_out/r03_$TAG
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1
tail -3 $O/pytest_gpu.log
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
cat $O/bench.json
for cfg in "$@"; do
  timeout -k 10 300 python bench.py --config $cfg > $O/bench_$cfg.json 2> $O/bench_$cfg.err
  cat $O/bench_$cfg.json
done
