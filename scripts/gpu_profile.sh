# rocprofv3 evidence for one bench workload (run on the GPU box through gpurun):
#   bash scripts/gpu_profile.sh <workload> <steps> [pmc]
# pass 1: --kernel-trace --stats (per-kernel durations); with "pmc": two further passes with
# FETCH_SIZE and WRITE_SIZE (separate passes: TCC slots), kernel-trace only.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
W=${1:-egnn}
S=${2:-5}
D=gpurun_out/prof_$W
mkdir -p $D
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o stats -- \
  python3 bench.py --workload $W --steps $S --warmup 1 --no-cpu-baseline --no-f32-exact --no-forward > $D/bench_stats.log 2>&1 || exit $?
if [ "${3:-}" = "pmc" ]; then
  timeout -k 10 900 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $D -o fetch -- \
    python3 bench.py --workload $W --steps 2 --warmup 1 --no-cpu-baseline --no-f32-exact --no-forward > $D/bench_fetch.log 2>&1 || exit $?
  timeout -k 10 900 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $D -o write -- \
    python3 bench.py --workload $W --steps 2 --warmup 1 --no-cpu-baseline --no-f32-exact --no-forward > $D/bench_write.log 2>&1 || exit $?
fi
find $D -name "*.csv" | sed -n 1,20p
