# Kernel trace of the MACE (or $W) bench under the given environment settings, then the stream
# overlap of the S kernel (scripts/trace_overlap.py).  Own time limit per GPU step.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for kv in "$@"; do export "$kv"; done
W=${W:-mace}
D=gpurun_out/trace_$W
mkdir -p $D
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $D -o t -- python3 bench.py --workload $W --steps 1 --warmup 1 --no-cpu-baseline > $D/bench.log 2>&1 || exit $?
python3 scripts/trace_overlap.py $D/t_kernel_trace.csv tp_node_outer > $D/overlap.txt 2>&1 || exit $?
cat $D/overlap.txt
