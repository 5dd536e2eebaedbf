# A/B benches (one process each, own time limit) + an EGNN kernel trace for the step timeline.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
if [ -n "${GMP_TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest $GMP_TESTS -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/ab/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc" >> gpurun_out/ab/pytest.log; tail -3 gpurun_out/ab/pytest.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
i=0
for args in "$@"; do
  i=$((i+1))
  timeout -k 10 300 python bench.py --no-cpu-baseline $args > gpurun_out/ab/bench_$i.log 2>&1 || exit $?
  echo "[$args] $(tail -1 gpurun_out/ab/bench_$i.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(round(d["value"]), round(d["ms_per_step"],2), d["config"].get("blas"), {k: round(v["value"]) for k,v in d.items() if isinstance(v, dict) and "value" in v and k!="cpu_baseline"})')"
done
if [ "${GMP_TRACE:-0}" = "1" ]; then
  mkdir -p gpurun_out/trace_egnn
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_egnn -o t -- python3 bench.py --workload egnn --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/trace_egnn/bench.log 2>&1 || exit $?
fi
