# Infinity-Cache sub-chunk experiment (scripts/mb_mall.py), then the r06 check pass.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u scripts/mb_mall.py 3 > gpurun_out/mb_mall.log 2>&1 || { cat gpurun_out/mb_mall.log; exit 1; }
cat gpurun_out/mb_mall.log
bash scripts/gpu_r06_check.sh
