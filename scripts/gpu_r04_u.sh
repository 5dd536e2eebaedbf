#!/bin/bash
# A/B: K4 HF planes at d + 16 halfs per row (default build) vs d + 8 (gmp_amd/ab/libgmp.so)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
AB=$PWD/geometric-message-passing_amd/gmp_amd/ab/libgmp.so
for r in 1 2 3; do
  for v in new old; do
    if [ $v = old ]; then export GMP_LIB=$AB; else unset GMP_LIB; fi
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-f32-exact --workload egnn > gpurun_out/ab/u_$v$r.log 2>&1 || exit $?
    echo "$v $(tail -1 gpurun_out/ab/u_$v$r.log | grep -o '"ms_per_step": [0-9.]*' | head -1) $(tail -1 gpurun_out/ab/u_$v$r.log | grep -o '"forward": {"edges_per_s": [0-9.]*')"
  done
done
