# Quick EGNN iteration on the GPU box: EGNN GPU parity tests + default bench (+ optional
# rocprofv3 kernel stats with GMP_PROFILE=1).  Each GPU step has its own time limit.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_egnn.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/egnn_tests.log 2>&1 || { tail -30 gpurun_out/egnn_tests.log; exit 1; }
tail -2 gpurun_out/egnn_tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/egnn_bench.log 2>&1 || { tail -30 gpurun_out/egnn_bench.log; exit 1; }
tail -1 gpurun_out/egnn_bench.log
if [ "${GMP_PROFILE:-0}" = "1" ]; then
  rm -rf gpurun_out/prof_iter
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_iter -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/prof_iter.log 2>&1 || exit 1
  f=$(find gpurun_out/prof_iter -name '*kernel_stats.csv' | head -1); python -c "import csv,sys; r=list(csv.DictReader(open('$f'))); [print(f\"{float(x['AverageNs'])/1e3:9.1f}us x{x['Calls']:>4} {float(x['Percentage']):5.1f}% {x['Name'][:90]}\") for x in r[:25]]"
fi
