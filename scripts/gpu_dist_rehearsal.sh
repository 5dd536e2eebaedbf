# Multi-process bench rehearsal on one GPU: two ranks over gloo run the default bench line
# (EGNN + MACE), the driver's N > 1 launch form with the collective backend swapped.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/dist
GMP_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/dist/bench2.log 2>&1 || { tail -20 gpurun_out/dist/bench2.log; exit 1; }
tail -1 gpurun_out/dist/bench2.log | cut -c1-600
