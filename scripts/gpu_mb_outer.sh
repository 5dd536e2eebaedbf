# S-kernel (tp_node_outer) at the full C4 shape, XCD-contiguous order on / off, then the MACE bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/mb
for x in 1 0; do
  for wd in 640 384; do
    GMP_TP_OUTER_XCD=$x C=50000 W=$wd OUTER_ONLY=1 timeout -k 10 120 python3 scripts/microbench_tpnode.py > gpurun_out/mb/outer_x${x}_w${wd}.log 2>&1 || exit $?
    echo "xcd=$x w=$wd $(tail -1 gpurun_out/mb/outer_x${x}_w${wd}.log)"
  done
done
timeout -k 10 300 python3 bench.py --workload mace --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/mb/mace.log 2>&1 || exit $?
tail -1 gpurun_out/mb/mace.log | cut -c1-400
