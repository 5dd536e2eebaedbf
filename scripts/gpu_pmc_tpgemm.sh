# SQ counters of the K7g kernels at the MACE-128 lo = 2 shape (one rocprofv3 pass, 8 SQ counters).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES --kernel-trace --output-format csv -d gpurun_out/pmc -o sq -- python3 scripts/mb_tpgemm.py 1 > gpurun_out/pmc/sq.log 2>&1 || exit $?
ls gpurun_out/pmc
