# One rocprofv3 SQ-counter pass (8 SQ counters) over a command: PMC_OUT names the output dir under
# gpurun_out/pmc; the table of per-kernel totals goes to <dir>/sq_table.md.
#   PMC_OUT=name bash scripts/gpu_pmc_cmd.sh python3 scripts/mb_tpfwd.py 1 5
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
D=gpurun_out/pmc/${PMC_OUT:-run}
mkdir -p $D
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES --kernel-trace --output-format csv -d $D -o sq -- "$@" > $D/run.log 2>&1 || exit $?
F=$(find $D -name "*counter_collection.csv" | head -n 1)
python3 scripts/sq_table.py "$F" > $D/sq_table.md || exit $?
cat $D/sq_table.md
