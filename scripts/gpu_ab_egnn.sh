# EGNN A/B: the EGNN GPU tests on the tree's build, then alternating bench lines (EGNN only) of
# the tree and abvar/old.  Own limit per step.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
timeout -k 10 600 python -u -m pytest tests/test_gpu_egnn.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/ab/pytest_egnn.log 2>&1 || { tail -30 gpurun_out/ab/pytest_egnn.log; exit 1; }
tail -2 gpurun_out/ab/pytest_egnn.log
for i in 1 2; do for v in tree old; do
  if [ $v = tree ]; then unset GMP_LIB GMP_TORCH_LIB; else export GMP_LIB=abvar/$v/libgmp.so GMP_TORCH_LIB=abvar/$v/libgmp_torch.so; fi
  timeout -k 10 300 python bench.py --workload egnn --steps 20 --warmup 3 --no-cpu-baseline --no-f32-exact --no-forward > gpurun_out/ab/egnn_$v$i.log 2>&1 || { tail -5 gpurun_out/ab/egnn_$v$i.log; exit 1; }
  echo "egnn $v: $(python3 -c "import json; d=json.loads(open('gpurun_out/ab/egnn_$v$i.log').read().strip().splitlines()[-1]); print(round(d['value']/1e6,2), 'M', round(d['ms_per_step'],3), 'ms', round(d['roofline']['ms_per_launch']*1e3,1), 'us bwd')")"
done; done
