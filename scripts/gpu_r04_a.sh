# r04 checkpoint: targeted GPU tests (GMP_TESTS), the K7s microbenchmark, then the EGNN trace.
# Every GPU step has its own time limit; a failure ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest ${GMP_TESTS:-tests} -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_some.log 2>&1 || { tail -40 gpurun_out/pytest_some.log; exit 1; }
tail -3 gpurun_out/pytest_some.log
timeout -k 10 300 python -u scripts/mb_tpfwd.py 3 5 3 > gpurun_out/mb_tpfwd.log 2>&1 || { cat gpurun_out/mb_tpfwd.log; exit 1; }
cat gpurun_out/mb_tpfwd.log
bash scripts/gpu_trace_egnn.sh
