# A/B of library builds on one box: GPU tests of the in-tree build (TESTS, optional), then
# bench.py for each "name:args" in $@ (name "tree" = the in-tree libraries, else abvar/<name>/).
# Every GPU step has its own time limit; a failure ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -x -q -m gpu --timeout 180 --timeout-method thread > gpurun_out/ab/pytest.log 2>&1 || { tail -40 gpurun_out/ab/pytest.log; exit 1; }
  tail -2 gpurun_out/ab/pytest.log
fi
i=0
for spec in "$@"; do
  i=$((i+1)); name=${spec%%:*}; args=${spec#*:}
  if [ "$name" = tree ]; then unset GMP_LIB GMP_TORCH_LIB
  else export GMP_LIB=abvar/$name/libgmp.so GMP_TORCH_LIB=abvar/$name/libgmp_torch.so; fi
  timeout -k 10 400 python bench.py --no-cpu-baseline $args > gpurun_out/ab/b$i.log 2>&1 || { tail -20 gpurun_out/ab/b$i.log; exit 1; }
  python3 scripts/ab_line.py gpurun_out/ab/b$i.log "$spec"
done
