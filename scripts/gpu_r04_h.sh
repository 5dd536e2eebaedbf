#!/bin/bash
# widening checks: K8 (D = 4 / 9 / 16, correlation 4), both-parity TP plans, boundary + ABI
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD/geometric-message-passing_amd
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_equivariant.py tests/test_gpu_boundary.py tests/test_abi.py \
  -k "symmetric or model_vs_oracle or boundary or abi or shape_checks or l3 or fused" \
  > gpurun_out/pytest_widen.log 2>&1; rc=$?
tail -30 gpurun_out/pytest_widen.log
exit $rc
