# r05 closing pass on the final tree: all GPU tests, smoke, default bench, GVP rocprofv3 evidence.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/gpu_round.sh || exit $?
bash scripts/gpu_profile.sh gvp 4 pmc > gpurun_out/prof_gvp.log 2>&1 || { tail gpurun_out/prof_gvp.log; exit 1; }
echo profile done
