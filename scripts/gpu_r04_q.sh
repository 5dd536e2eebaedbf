#!/bin/bash
# narrow-row LayerNorm kernels + GVP layer three-plane products: tests + GVP A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONPATH=$PWD/geometric-message-passing_amd
mkdir -p gpurun_out/ab
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_rowops.py tests/test_gpu_gvp.py > gpurun_out/pytest_q.log 2>&1 || { tail -30 gpurun_out/pytest_q.log; exit 1; }
tail -3 gpurun_out/pytest_q.log
for v in "GMP_GVP_X3=1" "GMP_GVP_X3=0" "GMP_LN_SMALL=0" "GMP_GVP_X3=1"; do
  env $v timeout -k 10 300 python bench.py --no-cpu-baseline --no-f32-exact --no-forward --workload gvp > gpurun_out/ab/q_$v.log 2>&1 || exit $?
  echo "$v $(tail -1 gpurun_out/ab/q_$v.log | cut -c150-260)"
done
