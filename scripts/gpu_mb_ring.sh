# Forward path GEMM A-ring depth sweep at the MACE-128 lo = 2 shape, node-form tests, MACE bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/mb
for r in 2 4 8; do
  GMP_TPGEMM_RING=$r timeout -k 10 180 python3 scripts/mb_tpgemm.py 5 fwd_gemm > gpurun_out/mb/ring$r.log 2>&1 || exit $?
  echo "ring=$r"; cat gpurun_out/mb/ring$r.log | grep -v amdgpu.ids
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_tpnode.py -x -q --timeout 300 --timeout-method thread > gpurun_out/mb/tpnode_tests.log 2>&1 || exit $?
tail -2 gpurun_out/mb/tpnode_tests.log
for r in 4 8; do
  GMP_TPGEMM_RING=$r timeout -k 10 300 python3 bench.py --workload mace --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/mb/mace_ring$r.log 2>&1 || exit $?
  echo "ring=$r $(tail -1 gpurun_out/mb/mace_ring$r.log | cut -c1-300)"
done
