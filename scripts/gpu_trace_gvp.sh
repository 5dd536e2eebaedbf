# Kernel trace of the GVP bench step under the given environment settings (VAR=value ...), then
# the per-stream timeline of one step (scripts/trace_timeline.py).  Own time limit per GPU step.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for kv in "$@"; do export "$kv"; done
D=gpurun_out/trace_gvp
mkdir -p $D
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $D -o t -- python3 bench.py --workload gvp --steps 3 --warmup 1 --no-cpu-baseline --no-f32-exact --no-forward > $D/bench.log 2>&1 || exit $?
F=$(find $D -name "*kernel_trace.csv" | head -n 1)
python3 scripts/trace_timeline.py "$F" gvp_msg0_fwd_kernel 4 -2 > $D/timeline.txt 2>&1 || exit $?
cat $D/timeline.txt | cut -c1-160
