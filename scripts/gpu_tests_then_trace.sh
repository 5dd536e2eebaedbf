# Targeted GPU tests (files given in GMP_TESTS), then the EGNN kernel trace + per-stream timeline.
# Every GPU step has its own time limit; a failure ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest ${GMP_TESTS:-tests} -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_some.log 2>&1 || { tail -30 gpurun_out/pytest_some.log; exit 1; }
tail -3 gpurun_out/pytest_some.log
bash scripts/gpu_trace_egnn.sh
