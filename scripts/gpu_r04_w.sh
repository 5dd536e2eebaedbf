#!/bin/bash
# GVP narrow products in four partial chains: tests + A/B against the previous build (gmp_amd/ab)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONPATH=$PWD/geometric-message-passing_amd
mkdir -p gpurun_out/ab
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_gvp.py > gpurun_out/pytest_w.log 2>&1 || { tail -30 gpurun_out/pytest_w.log; exit 1; }
tail -2 gpurun_out/pytest_w.log
AB=$PWD/geometric-message-passing_amd/gmp_amd/ab/libgmp.so
for r in 1 2; do
  for v in new old; do
    if [ $v = old ]; then export GMP_LIB=$AB; else unset GMP_LIB; fi
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-f32-exact --no-forward --workload gvp > gpurun_out/ab/w_$v$r.log 2>&1 || exit $?
    echo "$v $(tail -1 gpurun_out/ab/w_$v$r.log | grep -o '"ms_per_step": [0-9.]*' | head -1)"
  done
done
