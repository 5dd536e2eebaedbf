# SQ counter passes (one rocprofv3 --pmc run each, <= 8 SQ counters) over a command; per-kernel
# totals into gpurun_out/pmc/<PMC_OUT>/pass<i>.md.  A pass that errors (unknown counter) is
# reported and skipped; a pass killed at its time limit ends the script.
#   PMC_OUT=name bash scripts/gpu_pmc_passes.sh "CTR1 CTR2 .." "CTR .." -- python3 script.py
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
D=gpurun_out/pmc/${PMC_OUT:-run}
mkdir -p $D
passes=()
while [ "$1" != "--" ]; do passes+=("$1"); shift; done
shift
i=0
for ctrs in "${passes[@]}"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $ctrs --kernel-trace --output-format csv -d $D/p$i -o sq -- "$@" > $D/p$i.log 2>&1
  rc=$?
  if [ $rc -eq 137 ] || [ $rc -eq 124 ]; then echo "pass $i killed ($ctrs)"; exit $rc; fi
  if [ $rc -ne 0 ]; then echo "pass $i failed rc=$rc ($ctrs)"; tail -3 $D/p$i.log; continue; fi
  F=$(find $D/p$i -name "*counter_collection.csv" | head -n 1)
  python3 scripts/sq_raw.py "$F" egnn > $D/pass$i.md && cat $D/pass$i.md
done
