# TP A/B round 2: tests on the tree, T GEMM microbenchmark (tree vs abvar/zonly), then MACE / TFN
# bench lines of tree, abvar/zonly and abvar/old.  Own limit per step.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
timeout -k 10 900 python -u -m pytest tests/test_gpu_equivariant.py tests/test_gpu_tpnode.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/ab/pytest_tp.log 2>&1 || { tail -30 gpurun_out/ab/pytest_tp.log; exit 1; }
tail -1 gpurun_out/ab/pytest_tp.log
for v in tree zonly tree zonly; do
  if [ $v = tree ]; then unset GMP_LIB; else export GMP_LIB=abvar/$v/libgmp.so; fi
  echo "== $v"; timeout -k 10 300 python -u scripts/mb_tpgemm.py 5 T_gemm 2>&1 | grep T_gemm || exit 1
done
for w in mace tfn; do for v in tree zonly old tree zonly old; do
  if [ $v = tree ]; then unset GMP_LIB GMP_TORCH_LIB; else export GMP_LIB=abvar/$v/libgmp.so GMP_TORCH_LIB=abvar/$v/libgmp_torch.so; fi
  timeout -k 10 400 python bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline --no-f32-exact --no-forward > gpurun_out/ab/${w}_$v.log 2>&1 || { tail -5 gpurun_out/ab/${w}_$v.log; exit 1; }
  echo "$w $v: $(python3 -c "import json; d=json.loads(open('gpurun_out/ab/${w}_$v.log').read().strip().splitlines()[-1]); print(round(d['value']), round(d['ms_per_step'],1))")"
done; done
