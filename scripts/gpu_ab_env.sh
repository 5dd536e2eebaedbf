# A/B benches over environment settings: each argument is a space-separated list of VAR=value
# assignments ("" = defaults); BENCH_ARGS (default: --workload egnn) goes to every run.  One
# process per setting, each under its own time limit; a failure or timeout ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
BA=${BENCH_ARGS:-"--workload egnn"}
i=0
for spec in "$@"; do
  i=$((i+1))
  ( for kv in $spec; do export "$kv"; done
    timeout -k 10 400 python bench.py --no-cpu-baseline $BA > gpurun_out/ab/env_$i.log 2>&1 ) || exit $?
  echo "[$spec] $(tail -1 gpurun_out/ab/env_$i.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(round(d["value"]), round(d["ms_per_step"],2), {k: (round(v["value"]), round(v["ms_per_step"],1)) for k,v in d.items() if isinstance(v, dict) and "ms_per_step" in v})')"
done
