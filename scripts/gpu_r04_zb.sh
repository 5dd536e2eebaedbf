#!/bin/bash
# r04 closing call on the final tree: all GPU tests, smoke, default bench, TFN bench, then the
# GVP |vh| / vector-LayerNorm kernels A/B (GMP_GVP_VECNORM=1 vs 0) on the same box
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
bash scripts/gpu_r04_final.sh tests || exit $?
mkdir -p gpurun_out/ab
for v in 1 0; do
  GMP_GVP_VECNORM=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-f32-exact --no-forward --workload gvp > gpurun_out/ab/zb_$v.log 2>&1 || exit $?
  echo "fused=$v $(tail -1 gpurun_out/ab/zb_$v.log | grep -o '"ms_per_step": [0-9.]*' | head -1)"
done
