# Round-4 closing evidence, in two gpurun calls (each within the 20-minute call limit):
#   bash scripts/gpu_r04_final.sh tests     # full GPU tests, smoke, default bench line
#   bash scripts/gpu_r04_final.sh prof W    # kernel trace + PMC (FETCH_SIZE, WRITE_SIZE) of W
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
case "$1" in
  tests)
    GMP_BENCH=1 bash scripts/gpu_round.sh || exit $?
    timeout -k 10 600 python bench.py --workload tfn --steps 3 --warmup 1 > gpurun_out/bench_tfn.log 2>&1 || exit $?
    tail -1 gpurun_out/bench_tfn.log | cut -c1-400
    ;;
  prof)
    W=$2; S=2; [ "$W" = "egnn" ] && S=5
    bash scripts/gpu_profile.sh $W $S pmc > gpurun_out/prof_$W.log 2>&1 || exit $?
    python3 scripts/prof_summary.py gpurun_out/prof_$W $W r04 $((S + 1)) > /dev/null || exit $?
    head -n 14 profiles/r04_${W}_kernels.md
    ;;
esac
