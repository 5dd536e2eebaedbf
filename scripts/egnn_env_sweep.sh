# EGNN bench under several values of one environment knob (GPU box via gpurun):
#   VAR=GMP_SIDE_GRID_CAP VALUES="0 128" bash scripts/egnn_env_sweep.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in $VALUES; do
  env $VAR=$v timeout -k 10 240 python bench.py --workload ${WL:-egnn} --no-cpu-baseline --steps ${STEPS:-20} --warmup 3 ${BENCH_ARGS:-} > gpurun_out/sweep_$v.log 2>&1 || { tail -20 gpurun_out/sweep_$v.log; exit 1; }
  python -c "import json,sys; d=json.loads([l for l in open('gpurun_out/sweep_$v.log') if l.startswith('{')][-1]); print('$VAR=$v', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],3), 'ms')"
done
