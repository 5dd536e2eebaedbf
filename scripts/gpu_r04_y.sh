#!/bin/bash
# GVP vector LayerNorm kernels: tests (kernel, GVP suite, boundary incl. torch.compile), A/B bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONPATH=$PWD/geometric-message-passing_amd
mkdir -p gpurun_out/ab
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_gvp.py tests/test_gpu_boundary.py tests/test_abi.py > gpurun_out/pytest_y.log 2>&1 || { tail -30 gpurun_out/pytest_y.log; exit 1; }
tail -2 gpurun_out/pytest_y.log
for r in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-f32-exact --no-forward --workload gvp > gpurun_out/ab/y_$r.log 2>&1 || exit $?
  echo "new $(tail -1 gpurun_out/ab/y_$r.log | grep -o '"ms_per_step": [0-9.]*' | head -1)"
done
