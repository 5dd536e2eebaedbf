# K4 r05 check: EGNN GPU tests with the in-tree build, then (if the tree
# passes) bench A/B against the HEAD build.  Each step time-limited.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
timeout -k 10 400 python -u -m pytest tests/test_gpu_egnn.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/ab/t_tree.log 2>&1; rt=$?
tail -3 gpurun_out/ab/t_tree.log
[ $rt -eq 0 ] || [ $rt -eq 1 ] || exit $rt
[ $rt -eq 0 ] || exit 1
bash scripts/gpu_ab_var.sh "tree:--workload egnn --steps 20 --warmup 5" "base:--workload egnn --steps 20 --warmup 5" "tree:--workload egnn --steps 20 --warmup 5" "base:--workload egnn --steps 20 --warmup 5"
