#!/bin/bash
# swizzled / re-strided MFMA operand images (GVP three-plane, K4 HF): tests, benches, SQ counters
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONPATH=$PWD/geometric-message-passing_amd
mkdir -p gpurun_out/ab
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_gvp.py tests/test_gpu_egnn.py > gpurun_out/pytest_s.log 2>&1 || { tail -30 gpurun_out/pytest_s.log; exit 1; }
tail -2 gpurun_out/pytest_s.log
for v in "GMP_GVP_X3=1" "GMP_GVP_X3=0"; do
  env $v timeout -k 10 300 python bench.py --no-cpu-baseline --no-f32-exact --no-forward --workload gvp > gpurun_out/ab/s_$v.log 2>&1 || exit $?
  echo "gvp $v $(tail -1 gpurun_out/ab/s_$v.log | cut -c150-230)"
done
for r in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-f32-exact --workload egnn > gpurun_out/ab/s_egnn$r.log 2>&1 || exit $?
  echo "egnn $(tail -1 gpurun_out/ab/s_egnn$r.log | cut -c150-230) $(tail -1 gpurun_out/ab/s_egnn$r.log | grep -o '"forward": {[^}]*' | cut -c1-200)"
done
PMC_OUT=gvp2 bash scripts/gpu_pmc_cmd.sh python3 bench.py --workload gvp --steps 2 --warmup 1 --no-cpu-baseline --no-f32-exact --no-forward > /dev/null || exit $?
grep "gvp_" gpurun_out/pmc/gvp2/sq_table.md
PMC_OUT=egnn2 bash scripts/gpu_pmc_cmd.sh python3 bench.py --workload egnn --steps 2 --warmup 1 --no-cpu-baseline --no-f32-exact > /dev/null || exit $?
grep "egnn_" gpurun_out/pmc/egnn2/sq_table.md
