# K7 A/B: node-form tests on the tree's build, apply / T GEMM microbenchmarks (tree vs
# abvar/old), then the MACE (and optionally TFN) bench lines of both builds.  Own limit per step.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_tpnode.py -x -q -m gpu --timeout 120 --timeout-method thread 2>&1 | tail -3 || exit 1
mb() {  # name only
  if [ "$1" = tree ]; then unset GMP_LIB GMP_TORCH_LIB; else export GMP_LIB=abvar/$1/libgmp.so GMP_TORCH_LIB=abvar/$1/libgmp_torch.so; fi
  echo "== $1 $2"
  timeout -k 10 300 python -u scripts/mb_tpgemm.py 5 $2 2>&1 | grep -v amdgpu.ids || return 1
}
mb tree apply && mb old apply && mb tree T_gemm || exit 1
for w in ${WORKLOADS:-mace}; do
  for v in tree old; do
    if [ "$v" = tree ]; then unset GMP_LIB GMP_TORCH_LIB; else export GMP_LIB=abvar/$v/libgmp.so GMP_TORCH_LIB=abvar/$v/libgmp_torch.so; fi
    timeout -k 10 400 python bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline --no-f32-exact --no-forward > gpurun_out/ab_k7_$w_$v.log 2>&1 || { tail -20 gpurun_out/ab_k7_$w_$v.log; exit 1; }
    echo "$w $v: $(python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab_k7_$w_$v.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])")"
  done
done
