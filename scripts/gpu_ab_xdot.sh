# xyz-dot sums: GPU tests, then alternating bench runs with and without them (one box).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
timeout -k 10 400 python -u -m pytest tests/test_gpu_gvp.py -x -q --timeout 180 --timeout-method thread > gpurun_out/t_gvp.log 2>&1 || { tail -30 gpurun_out/t_gvp.log; exit 3; }
tail -1 gpurun_out/t_gvp.log
G="--workload gvp --steps 10 --warmup 3 --no-cpu-baseline --no-f32-exact --no-forward"
for i in 1 2; do
  timeout -k 10 300 python bench.py $G > gpurun_out/ab/x_on$i.log 2>&1 || exit 1
  python3 scripts/ab_line.py gpurun_out/ab/x_on$i.log on
  timeout -k 10 300 python scripts/ab_xyz_dot_off.py $G > gpurun_out/ab/x_off$i.log 2>&1 || exit 1
  python3 scripts/ab_line.py gpurun_out/ab/x_off$i.log off
done
