# TP tests + rocprofv3 kernel stats of a short MACE bench (GPU box; via gpurun).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_mace
timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_gpu_tpnode.py tests/test_gpu_equivariant.py} -m gpu --timeout 200 --timeout-method thread -q > gpurun_out/tp.log 2>&1
rc=$?; tail -3 gpurun_out/tp.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_mace -o stats -- python3 bench.py --workload mace --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof_mace/bench.log 2>&1 || exit $?
tail -1 gpurun_out/prof_mace/bench.log | cut -c1-400
