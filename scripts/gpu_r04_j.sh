#!/bin/bash
# K8 rolled-only build: symmetric-contraction tests + timing, then an EGNN side-stream A/B
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD/geometric-message-passing_amd
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_equivariant.py -k "symmetric or mace_c4_config or model_vs_oracle" > gpurun_out/pytest_sc.log 2>&1 || { tail -30 gpurun_out/pytest_sc.log; exit 1; }
tail -2 gpurun_out/pytest_sc.log
timeout -k 10 120 python -u scripts/mb_sc.py > gpurun_out/mb_sc.log 2>&1 && cat gpurun_out/mb_sc.log
