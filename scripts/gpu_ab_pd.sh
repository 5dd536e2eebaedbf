# A/B of the weight-sum kernel's NL = 2 ring depth (abvar/pd3) against the tree: the GVP tests
# on the variant, the 128 x 144 edge outer sum, then the GVP bench line, alternating.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
V=${V:-pd3}
GMP_LIB=abvar/$V/libgmp.so GMP_TORCH_LIB=abvar/$V/libgmp_torch.so timeout -k 10 600 python -u -m pytest tests/test_gpu_gvp.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/ab/pytest_$V.log 2>&1 || { tail -30 gpurun_out/ab/pytest_$V.log; exit 1; }
tail -1 gpurun_out/ab/pytest_$V.log
for v in tree $V tree $V; do
  if [ $v = tree ]; then unset GMP_LIB GMP_TORCH_LIB; else export GMP_LIB=abvar/$v/libgmp.so GMP_TORCH_LIB=abvar/$v/libgmp_torch.so; fi
  echo "== $v"; timeout -k 10 300 python -u scripts/microbench_wgrad.py 2>&1 | grep "128x144" || exit 1
done
for v in tree $V tree $V; do
  if [ $v = tree ]; then unset GMP_LIB GMP_TORCH_LIB; else export GMP_LIB=abvar/$v/libgmp.so GMP_TORCH_LIB=abvar/$v/libgmp_torch.so; fi
  timeout -k 10 400 python bench.py --workload gvp --steps 10 --warmup 2 --no-cpu-baseline --no-f32-exact --no-forward > gpurun_out/ab/gvp_$v.log 2>&1 || { tail -5 gpurun_out/ab/gvp_$v.log; exit 1; }
  echo "gvp $v: $(python3 -c "import json; d=json.loads(open('gpurun_out/ab/gvp_$v.log').read().strip().splitlines()[-1]); print(round(d['value']), round(d['ms_per_step'],2))")"
done
