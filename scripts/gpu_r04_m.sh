#!/bin/bash
# dW2p store permutation (XOR 1) + EGNN edge-sum side lane: tests, dW2p SQ pass, EGNN A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD/geometric-message-passing_amd
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_tpnode.py tests/test_gpu_wgrad.py tests/test_gpu_egnn.py tests/test_gpu_dist.py > gpurun_out/pytest_m.log 2>&1 || { tail -20 gpurun_out/pytest_m.log; exit 1; }
tail -2 gpurun_out/pytest_m.log
PMC_OUT=k7c bash scripts/gpu_pmc_cmd.sh python3 scripts/mb_tpgemm.py 1 dW > /dev/null || exit $?
grep -E "outer_cols" gpurun_out/pmc/k7c/sq_table.md; grep " ms " gpurun_out/pmc/k7c/run.log
BENCH_ARGS="--workload egnn --no-f32-exact --no-forward" bash scripts/gpu_ab_env.sh "" "GMP_EDGE_SUM_LANE=0" "" "GMP_EDGE_SUM_LANE=0"
