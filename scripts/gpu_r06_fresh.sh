# The bench line with a fresh edge_index tensor per step (K0's CSR build inside every timed
# step, as the reference's loader-fed step) beside the cached-graph line, on one box.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python bench.py --fresh-graph --no-cpu-baseline > gpurun_out/bench_fresh.log 2>&1 || { tail -5 gpurun_out/bench_fresh.log; exit 1; }
tail -1 gpurun_out/bench_fresh.log | cut -c1-300
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench_cached.log 2>&1 || { tail -5 gpurun_out/bench_cached.log; exit 1; }
tail -1 gpurun_out/bench_cached.log | cut -c1-300
