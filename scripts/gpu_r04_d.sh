# Unit tests of the r04 kernels, K7s microbench + SQ counters, EGNN A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_wgrad.py tests/test_gpu_tpnode.py tests/test_gpu_rowops.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_some.log 2>&1 || { tail -40 gpurun_out/pytest_some.log; exit 1; }
tail -2 gpurun_out/pytest_some.log
timeout -k 10 300 python -u scripts/mb_tpfwd.py 3 5 3 > gpurun_out/mb_tpfwd.log 2>&1 || { cat gpurun_out/mb_tpfwd.log; exit 1; }
cat gpurun_out/mb_tpfwd.log
PMC_OUT=k7s bash scripts/gpu_pmc_cmd.sh python3 scripts/mb_tpfwd.py 1 5 | grep -E "kernel|fused|outer_kernel|gemm_x3" || exit $?
BENCH_ARGS="--workload egnn --no-f32-exact --no-forward" bash scripts/gpu_ab_env.sh "" "GMP_WGRAD_QUAD=0" "GMP_LN_R03=1" "GMP_WGRAD_QUAD=0 GMP_LN_R03=1" ""
