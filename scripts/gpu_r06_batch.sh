# r06 batch: EGNN A/B (tests + alternating bench lines), the equivariant GPU tests and MACE / TFN
# profiles (kernel trace + PMC passes), then the EGNN SQ-counter pass.  Own limit per step.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/gpu_ab_egnn.sh || exit $?
unset GMP_LIB GMP_TORCH_LIB
bash scripts/gpu_r06_mace.sh || exit $?
PMC_OUT=egnn_sq bash scripts/gpu_pmc_passes.sh "SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES" -- python3 bench.py --workload egnn --steps 2 --warmup 1 --no-cpu-baseline --no-f32-exact --no-forward > gpurun_out/egnn_sq.log 2>&1 || { tail gpurun_out/egnn_sq.log; exit 1; }
F=$(find gpurun_out/pmc/egnn_sq/p1 -name "*counter_collection.csv" | head -n 1)
python3 scripts/sq_table.py "$F" > gpurun_out/egnn_sq_table.md && head -12 gpurun_out/egnn_sq_table.md
