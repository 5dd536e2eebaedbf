#!/bin/bash
# A/B on one box: GVP vector LayerNorm kernel (GMP_GVP_VECNORM=1) vs the torch chain (=0)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
for r in 1 2; do
  for v in 1 0; do
    GMP_GVP_VECNORM=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-f32-exact --no-forward --workload gvp > gpurun_out/ab/z_$v$r.log 2>&1 || exit $?
    echo "vecnorm=$v $(tail -1 gpurun_out/ab/z_$v$r.log | grep -o '"ms_per_step": [0-9.]*' | head -1)"
  done
done
