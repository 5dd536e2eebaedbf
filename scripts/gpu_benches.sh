# GPU suite + bench lines for several workloads (each step time-limited; stops at the first
# failure).  usage: bash scripts/gpu_benches.sh "egnn gvp" [tests]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${2:-}" = "tests" ]; then
  timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
  tail -1 gpurun_out/pytest_gpu.log
fi
for W in ${1:-egnn}; do
  S=10; [ "$W" = "mace" ] && S=2; [ "$W" = "tfn" ] && S=2; [ "$W" = "gvp" ] && S=5
  timeout -k 10 600 python bench.py --workload $W --steps $S --warmup 2 ${BENCH_ARGS:---no-cpu-baseline} > gpurun_out/bench_$W.log 2>&1 || { tail -20 gpurun_out/bench_$W.log; exit 1; }
  tail -1 gpurun_out/bench_$W.log | cut -c1-400
done
