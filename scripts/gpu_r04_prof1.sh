#!/bin/bash
# r04 profiles, part 1: EGNN and GVP kernel traces + HBM passes, then the K7 SQ counter passes
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD/geometric-message-passing_amd
bash scripts/gpu_r04_final.sh prof egnn || exit $?
bash scripts/gpu_r04_final.sh prof gvp || exit $?
PMC_OUT=k7 bash scripts/gpu_pmc_cmd.sh python3 scripts/mb_tpgemm.py 1 || exit $?
PMC_OUT=k7s bash scripts/gpu_pmc_cmd.sh python3 scripts/mb_tpfwd.py 1 5 || exit $?
