# r06: the equivariant GPU tests (MACE / TFN node form incl. the C4 / C5 configs vs the oracle),
# then rocprofv3 kernel traces + PMC passes of the MACE and TFN bench workloads.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_equivariant.py tests/test_gpu_tpnode.py -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_eq.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_eq.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_profile.sh mace 2 pmc > gpurun_out/prof_mace.log 2>&1 || { tail gpurun_out/prof_mace.log; exit 1; }
bash scripts/gpu_profile.sh tfn 2 pmc > gpurun_out/prof_tfn.log 2>&1 || { tail gpurun_out/prof_tfn.log; exit 1; }
echo profiles done
