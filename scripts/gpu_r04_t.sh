#!/bin/bash
# r04 closing, second call: the multi-rank GPU tests again, then EGNN / GVP kernel profiles
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_dist.log 2>&1 || { tail -20 gpurun_out/pytest_dist.log; exit 1; }
tail -2 gpurun_out/pytest_dist.log
bash scripts/gpu_r04_final.sh prof gvp || exit $?
bash scripts/gpu_r04_final.sh prof egnn || exit $?
