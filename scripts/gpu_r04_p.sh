#!/bin/bash
# eager vs HIP-graph replay for GVP / EGNN / TFN
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
for w in gvp egnn; do
  for g in "" "--graph"; do
    timeout -k 10 400 python bench.py --no-cpu-baseline --no-f32-exact --no-forward --workload $w $g > gpurun_out/ab/graph_${w}${g}.log 2>&1 || exit $?
    echo "$w $g $(tail -1 gpurun_out/ab/graph_${w}${g}.log | cut -c1-200)"
  done
done
