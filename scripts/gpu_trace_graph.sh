# EGNN step timeline under HIP-graph replay vs eager (kernel trace per stream)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for mode in eager graph; do
  mkdir -p gpurun_out/trace_$mode
  extra=""; [ $mode = graph ] && extra="--graph"
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_$mode -o t -- python3 bench.py --workload egnn --steps 3 --warmup 1 --no-cpu-baseline $extra > gpurun_out/trace_$mode/bench.log 2>&1 || exit $?
  f=$(find gpurun_out/trace_$mode -name "*kernel_trace.csv" | head -n 1)
  idx=-2; [ $mode = graph ] && idx=-4
  python3 scripts/trace_timeline.py $f egnn_fwd_kernel 4 $idx > gpurun_out/trace_$mode/timeline.txt || exit $?
  echo "== $mode"; head -n 40 gpurun_out/trace_$mode/timeline.txt
done
