# A/B of eager vs HIP-graph replay of the training step (bench.py --graph), EGNN and GVP.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/ab_graph
mkdir -p $D
for w in egnn gvp; do
  for mode in "" "--graph" "" "--graph"; do
    timeout -k 10 300 python3 bench.py --workload $w --steps 20 --warmup 3 --no-cpu-baseline --no-f32-exact --no-forward $mode > $D/b.json 2> $D/b.err || exit $?
    python3 -c "import json,sys; d=json.loads(open('$D/b.json').read().strip().splitlines()[-1]); o=d if '$w'=='egnn' else d.get('$w', d); print('$w', '$mode' or 'eager', round(o.get('value', 0)/1e6, 2), 'M', round(o.get('ms_per_step', 0), 3), 'ms')"
  done
done
