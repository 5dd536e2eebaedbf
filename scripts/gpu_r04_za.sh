#!/bin/bash
# GVP |vh| kernel: tests (GVP suite, boundary incl. torch.compile, ABI), A/B with the torch chains
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONPATH=$PWD/geometric-message-passing_amd
mkdir -p gpurun_out/ab
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_gvp.py tests/test_gpu_boundary.py tests/test_abi.py > gpurun_out/pytest_za.log 2>&1 || { tail -30 gpurun_out/pytest_za.log; exit 1; }
tail -2 gpurun_out/pytest_za.log
for r in 1 2; do
  for v in 1 0; do
    GMP_GVP_VECNORM=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-f32-exact --no-forward --workload gvp > gpurun_out/ab/za_$v$r.log 2>&1 || exit $?
    echo "fused=$v $(tail -1 gpurun_out/ab/za_$v$r.log | grep -o '"ms_per_step": [0-9.]*' | head -1)"
  done
done
