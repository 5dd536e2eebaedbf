# Outer-sum LDS row permutation: unit tests of every outer-sum entry point, the dW2p kernel at the
# MACE lo = 2 shape (time + bank-conflict counter), EGNN and MACE benches.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/perm
timeout -k 10 600 python -u -m pytest tests/test_gpu_wgrad.py tests/test_gpu_tpnode.py tests/test_gpu_egnn.py tests/test_gpu_gvp.py tests/test_gpu_equivariant.py -x -q --timeout 300 --timeout-method thread > gpurun_out/perm/tests.log 2>&1 || { tail -30 gpurun_out/perm/tests.log; exit 1; }
tail -1 gpurun_out/perm/tests.log
timeout -k 10 240 python3 scripts/mb_tpgemm.py 3 > gpurun_out/perm/dw.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/perm/dw.log
timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_INSTS_VALU --kernel-trace --output-format csv -d gpurun_out/perm -o sq -- python3 scripts/mb_tpgemm.py 1 dW > gpurun_out/perm/sq.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --workload egnn --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/perm/egnn.log 2>&1 || exit $?
echo "egnn $(tail -1 gpurun_out/perm/egnn.log | cut -c1-200)"
timeout -k 10 300 python3 bench.py --workload mace --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/perm/mace.log 2>&1 || exit $?
echo "mace $(tail -1 gpurun_out/perm/mace.log | cut -c1-200)"
