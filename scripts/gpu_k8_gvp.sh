# K8 tests + microbench, then a kernel trace of the GVP step (per-stream busy time).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_equivariant.py -k "symmetric or mace" tests/test_gpu_boundary.py > gpurun_out/k8.log 2>&1 || { tail -30 gpurun_out/k8.log; exit 1; }
tail -3 gpurun_out/k8.log
timeout -k 10 300 python -u scripts/mb_sc.py > gpurun_out/mb_sc.log 2>&1 || exit $?
cat gpurun_out/mb_sc.log
D=gpurun_out/trace_gvp
mkdir -p $D
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $D -o t -- python3 bench.py --workload gvp --steps 3 --warmup 1 --no-cpu-baseline --no-forward > $D/bench.log 2>&1 || exit $?
F=$(find $D -name "*kernel_trace.csv" | head -n 1)
python3 scripts/trace_gaps.py "$F" gvp_msg0_fwd 700 4 > $D/gaps.txt 2>&1 || exit $?
tail -40 $D/gaps.txt | cut -c1-160
