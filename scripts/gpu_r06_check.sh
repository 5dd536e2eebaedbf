# r06 pass on the current tree: all GPU tests, smoke, default bench, then the EGNN kernel
# trace with the FETCH_SIZE / WRITE_SIZE passes. Every GPU step has its own limit.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/gpu_round.sh || exit $?
bash scripts/gpu_profile.sh egnn 5 pmc > gpurun_out/prof_egnn.log 2>&1 || { tail gpurun_out/prof_egnn.log; exit 1; }
echo profile done
