# Alternating A/B runs of one workload with a module attribute on / off:
#   bash scripts/gpu_ab_toggle.sh <workload> <module> <attr> [rounds] [steps]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for k in $(seq 1 ${4:-2}); do
  for v in 1 0; do
    timeout -k 10 400 python3 scripts/ab_toggle_bench.py $1 $2 $3 $v ${5:-20} || exit $?
  done
done
