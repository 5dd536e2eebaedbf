#!/bin/bash
# SQ counters of the EGNN (incl. the inference forward) and GVP kernels at the bench shapes
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
PMC_OUT=egnn bash scripts/gpu_pmc_cmd.sh python3 bench.py --workload egnn --steps 2 --warmup 1 --no-cpu-baseline --no-f32-exact > /dev/null || exit $?
PMC_OUT=gvp bash scripts/gpu_pmc_cmd.sh python3 bench.py --workload gvp --steps 2 --warmup 1 --no-cpu-baseline --no-f32-exact --no-forward > /dev/null || exit $?
head -n 30 gpurun_out/pmc/egnn/sq_table.md
head -n 30 gpurun_out/pmc/gvp/sq_table.md
