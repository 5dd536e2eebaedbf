# K8 GPU tests + microbench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_equivariant.py -k "symmetric or mace" tests/test_gpu_boundary.py > gpurun_out/k8.log 2>&1 || { tail -30 gpurun_out/k8.log; exit 1; }
tail -3 gpurun_out/k8.log
timeout -k 10 300 python -u scripts/mb_sc.py > gpurun_out/mb_sc.log 2>&1 || exit $?
cat gpurun_out/mb_sc.log
