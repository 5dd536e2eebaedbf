#!/bin/bash
# K7s: parity test, then spread and uniform in-degree timings
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD/geometric-message-passing_amd
timeout -k 10 120 python -u -m pytest -x -q --timeout 100 --timeout-method thread tests/test_gpu_tpnode.py -k fused > gpurun_out/pytest_fused.log 2>&1 && \
timeout -k 10 180 python -u scripts/mb_tpfwd.py 3 5 3 > gpurun_out/mb_tpfwd.log 2>&1 && \
GMP_TPF_DIAG=1 timeout -k 10 180 python -u scripts/mb_tpfwd.py 3 5 3 > gpurun_out/mb_diag1.log 2>&1; cat gpurun_out/pytest_fused.log gpurun_out/mb_tpfwd.log gpurun_out/mb_diag1.log
