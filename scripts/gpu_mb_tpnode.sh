set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/mb
timeout -k 10 120 python3 scripts/microbench_tpnode.py > gpurun_out/mb/tpnode.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES --kernel-trace --output-format csv -d gpurun_out/mb -o pmc1 -- python3 scripts/microbench_tpnode.py > gpurun_out/mb/pmc1.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/mb -o pmc2 -- python3 scripts/microbench_tpnode.py > gpurun_out/mb/pmc2.log 2>&1
