#!/bin/bash
# max_ell = 5 (SH l = 4, 5 in K1, runtime-l z / dz kernels): featurise + model tests vs oracle,
# then the equivariant suite
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD/geometric-message-passing_amd
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_equivariant.py \
  -k "featurize or model_vs_oracle" > gpurun_out/pytest_n.log 2>&1; rc=$?
tail -30 gpurun_out/pytest_n.log
exit $rc
