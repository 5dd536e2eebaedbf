#!/bin/bash
# K8 after the rolled-loop split: widening tests again, then the unrolled / rolled timing A/B
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD/geometric-message-passing_amd
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_equivariant.py -k "symmetric or model_vs_oracle" > gpurun_out/pytest_widen2.log 2>&1 || { tail -30 gpurun_out/pytest_widen2.log; exit 1; }
tail -2 gpurun_out/pytest_widen2.log
timeout -k 10 120 python -u scripts/mb_sc.py > gpurun_out/mb_sc.log 2>&1 && \
GMP_SC_ROLLED=1 timeout -k 10 120 python -u scripts/mb_sc.py >> gpurun_out/mb_sc.log 2>&1; cat gpurun_out/mb_sc.log
