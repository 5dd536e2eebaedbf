# Round check (GPU tests, smoke, default bench) followed by a kernel-trace profile of the EGNN
# and MACE bench workloads.  Every GPU step has its own time limit; a failure ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_round.sh || exit $?
NO_TESTS=1 bash scripts/gpu_profile.sh egnn 5 || exit $?
bash scripts/gpu_profile.sh mace 2 || exit $?
