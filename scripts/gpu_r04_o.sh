#!/bin/bash
# TP conv aggr max / min + the equivariant / boundary suites
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD/geometric-message-passing_amd
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_equivariant.py tests/test_gpu_boundary.py > gpurun_out/pytest_o.log 2>&1; rc=$?
tail -30 gpurun_out/pytest_o.log
exit $rc
