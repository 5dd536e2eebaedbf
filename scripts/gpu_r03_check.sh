# r03: the new / changed GPU tests, then rocprofv3 kernel-trace + PMC (FETCH_SIZE, WRITE_SIZE)
# summaries of the EGNN, MACE and TFN bench workloads.  Each GPU step has its own time limit;
# a failure or timeout ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${GMP_TESTS:-"tests/test_gpu_boundary.py tests/test_gpu_wgrad.py tests/test_gpu_gvp.py tests/test_gpu_dist.py tests/test_gpu_egnn.py::test_egnn_c2_full_size_properties_hf tests/test_gpu_equivariant.py::test_tfn_c5_collated_batch_equals_per_graph_sum"}
timeout -k 10 900 python -u -m pytest $T -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_r03.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_r03.log
tail -3 gpurun_out/pytest_r03.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if [ "${GMP_PROF:-1}" = "1" ]; then
  for W in ${GMP_PROF_W:-egnn mace tfn}; do
    S=2; [ "$W" = "egnn" ] && S=5
    bash scripts/gpu_profile.sh $W $S pmc > gpurun_out/prof_$W.log 2>&1 || exit $?
    tail -1 gpurun_out/prof_$W/bench_stats.log | cut -c1-300
  done
fi
