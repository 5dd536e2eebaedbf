# r06 closing pass on the final tree: all GPU tests, smoke, default bench, then rocprofv3 kernel
# traces + PMC passes of the GVP, MACE and TFN bench workloads.  Own limit per step.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/gpu_round.sh || exit $?
for w in gvp mace tfn; do
  S=2; [ $w = gvp ] && S=4
  bash scripts/gpu_profile.sh $w $S pmc > gpurun_out/prof_$w.log 2>&1 || { tail gpurun_out/prof_$w.log; exit 1; }
  echo "profile $w done"
done
