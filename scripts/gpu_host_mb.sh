# EGNN host-enqueue vs wall time (is the eager step host-bound?) and the K7 kernels at the
# MACE-128 lo = 2 shape.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/mb
FUSED=1 timeout -k 10 300 python3 scripts/host_profile.py egnn > gpurun_out/mb/host_egnn.log 2>&1 || exit $?
head -60 gpurun_out/mb/host_egnn.log | grep -v amdgpu.ids
timeout -k 10 300 python3 scripts/mb_tpgemm.py 3 > gpurun_out/mb/tpgemm_all.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/mb/tpgemm_all.log
