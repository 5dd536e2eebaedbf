# K7s (blocked z layout): unit test, microbench, SQ counters.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_tpnode.py -x -q -m gpu -k fwd_fused --timeout 120 --timeout-method thread > gpurun_out/pytest_some.log 2>&1 || { tail -40 gpurun_out/pytest_some.log; exit 1; }
tail -2 gpurun_out/pytest_some.log
timeout -k 10 300 python -u scripts/mb_tpfwd.py 3 5 3 > gpurun_out/mb_tpfwd.log 2>&1 || { cat gpurun_out/mb_tpfwd.log; exit 1; }
cat gpurun_out/mb_tpfwd.log
PMC_OUT=k7s bash scripts/gpu_pmc_cmd.sh python3 scripts/mb_tpfwd.py 1 5 | grep -E "kernel|fused|outer_kernel|gemm_x3" || exit $?
