# Path GEMM register-ring sweep (A / B streams) at the MACE-128 lo = 2 shape, then the MACE bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/mb
for cfg in "8 2" "8 4" "44 4"; do
  set -- $cfg
  GMP_TPGEMM_RING=$1 GMP_TPGEMM_WIDEN_RING=$2 timeout -k 10 240 python3 scripts/mb_tpgemm.py 3 gemm > gpurun_out/mb/rings_$1_$2.log 2>&1 || exit $?
  echo "ring=$1 widen=$2"; grep -v amdgpu.ids gpurun_out/mb/rings_$1_$2.log
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_tpnode.py -x -q --timeout 300 --timeout-method thread > gpurun_out/mb/tpnode_tests.log 2>&1 || exit $?
tail -1 gpurun_out/mb/tpnode_tests.log
timeout -k 10 300 python3 bench.py --workload mace --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/mb/mace_def.log 2>&1 || exit $?
echo "default $(tail -1 gpurun_out/mb/mace_def.log | cut -c1-260)"
