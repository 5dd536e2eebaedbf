#!/bin/bash
# tpnode / wgrad tests (K7g stagger default, dW2p permuted LDS rows), dW2p microbench, then the
# EGNN node-level quadrant-sum A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD/geometric-message-passing_amd
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_tpnode.py tests/test_gpu_wgrad.py > gpurun_out/pytest_q.log 2>&1 || { tail -20 gpurun_out/pytest_q.log; exit 1; }
tail -2 gpurun_out/pytest_q.log
timeout -k 10 300 python -u scripts/mb_tpgemm.py 5 > gpurun_out/mb_tpgemm_all.log 2>&1 && cat gpurun_out/mb_tpgemm_all.log || exit 1
BENCH_ARGS="--workload egnn --no-f32-exact --no-forward" bash scripts/gpu_ab_env.sh "" "GMP_QUAD_WG2=2" "GMP_QUAD_WG2=1" "GMP_QUAD_WG2=8" ""
