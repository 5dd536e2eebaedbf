# K7s SQ counters (microbench, lo = 2 shape) + EGNN stream-priority / LN-backward A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
PMC_OUT=k7s bash scripts/gpu_pmc_cmd.sh python3 scripts/mb_tpfwd.py 1 5 || exit $?
BENCH_ARGS="--workload egnn --no-f32-exact --no-forward" bash scripts/gpu_ab_env.sh "" "GMP_MAIN_STREAM=1" "GMP_MAIN_STREAM=1 GMP_MAIN_PRIO=1" "GMP_LN_R03=1" "GMP_MAIN_STREAM=1 GMP_MAIN_PRIO=1 GMP_LN_R03=1" ""
