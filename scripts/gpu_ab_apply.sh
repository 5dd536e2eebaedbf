# A/B in one process pair on one box: the apply kernels at the MACE lo = 2 shape with the
# conflict-free A staging (libgmp.so) against the previous staging (libgmp_alt.so), twice each.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
for i in 1 2; do
  for lib in libgmp.so libgmp_alt.so; do
    GMP_LIB=geometric-message-passing_amd/gmp_amd/$lib timeout -k 10 240 python3 scripts/mb_tpgemm.py 3 apply > gpurun_out/ab/$lib.$i.log 2>&1 || exit $?
    echo "$lib $(grep apply gpurun_out/ab/$lib.$i.log)"
  done
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_tpnode.py -x -q -k apply --timeout 300 --timeout-method thread > gpurun_out/ab/tests.log 2>&1 || exit $?
tail -1 gpurun_out/ab/tests.log
