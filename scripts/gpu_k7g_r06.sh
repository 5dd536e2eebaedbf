# r06 K7g round: diagnostics / A-B (scripts/gpu_diag_k7g.sh with the variant lists in the
# environment), then the MACE bench of the tree's build and of abvar/old.  Own limit per step.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/diag
L=gpurun_out/diag/${TAG:-k7g}.log
bash scripts/gpu_diag_k7g.sh > $L 2>&1 || { cat $L; exit 1; }
for v in ${BENCH_VARIANTS:-tree old}; do
  if [ $v = tree ]; then unset GMP_LIB GMP_TORCH_LIB; else export GMP_LIB=abvar/$v/libgmp.so GMP_TORCH_LIB=abvar/$v/libgmp_torch.so; fi
  for w in ${WORKLOADS:-mace}; do
    timeout -k 10 400 python bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline --no-f32-exact --no-forward > gpurun_out/diag/${w}_$v.log 2>&1 || { tail -5 gpurun_out/diag/${w}_$v.log; exit 1; }
    echo "$w $v $(tail -1 gpurun_out/diag/${w}_$v.log | cut -c1-150)" >> $L
  done
done
cat $L
