# K7g A/B at the MACE-128 lo = 2 shape (scripts/mb_tpgemm.py): the tree's build against
# abvar/<name>/libgmp.so variants, after the K7g GEMM tests on the tree.  Own limit per step.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_tpnode.py -x -q -m gpu --timeout 120 --timeout-method thread -k "widen or gemm" 2>&1 | tail -3 || exit 1
run() {  # name only
  if [ "$1" = tree ]; then unset GMP_LIB; else export GMP_LIB=abvar/$1/libgmp.so; fi
  echo "== $1 $2"
  timeout -k 10 300 python -u scripts/mb_tpgemm.py 5 $2 2>&1 | grep -v amdgpu.ids || return 1
}
for v in ${T_VARIANTS:-tree}; do run $v T_gemm || exit 1; done
for v in ${F_VARIANTS:-}; do run $v fwd_gemm || exit 1; done
for v in ${D_VARIANTS:-}; do run $v dW_cols || exit 1; done
