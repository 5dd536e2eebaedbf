# One GPU-box pass: GPU tests (all, not stopping at the first failure), smoke, default bench.
# Every GPU step has its own time limit; a timeout / crash ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TESTS:-tests}
timeout -k 10 900 python -u -m pytest $T -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
cat gpurun_out/smoke.log | grep smoke
if [ "${BENCH:-1}" = "1" ]; then
  timeout -k 10 900 python bench.py > gpurun_out/bench.log 2>&1 || exit $?
  tail -1 gpurun_out/bench.log
fi
