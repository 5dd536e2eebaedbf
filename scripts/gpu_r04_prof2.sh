#!/bin/bash
# r04 profiles, part 2: MACE and TFN kernel traces + HBM passes, then the K7 SQ pass again
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD/geometric-message-passing_amd
bash scripts/gpu_r04_final.sh prof mace || exit $?
PMC_OUT=k7b bash scripts/gpu_pmc_cmd.sh python3 scripts/mb_tpgemm.py 1 || exit $?
bash scripts/gpu_r04_final.sh prof tfn || exit $?
