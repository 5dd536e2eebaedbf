#!/bin/bash
# GVP layer backward without spre rows + K7g forward B buffer loads: GPU tests, GEMM A/B
# (static priority for waves 4-7), GVP bench
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD/geometric-message-passing_amd
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_gvp.py tests/test_gpu_tpnode.py tests/test_gpu_boundary.py tests/test_abi.py \
  > gpurun_out/pytest_k.log 2>&1 || { tail -30 gpurun_out/pytest_k.log; exit 1; }
tail -2 gpurun_out/pytest_k.log
timeout -k 10 300 python -u scripts/mb_tpgemm.py 5 gemm > gpurun_out/mb_tpgemm.log 2>&1 && \
GMP_GEMM_PRIO=1 timeout -k 10 300 python -u scripts/mb_tpgemm.py 5 gemm >> gpurun_out/mb_tpgemm.log 2>&1 && cat gpurun_out/mb_tpgemm.log
