# r05 closing pass: the K1e tests first (a failure ends the script), the K1e microbenchmark, then
# the round check (all GPU tests, smoke, default bench) and the GVP rocprofv3 evidence.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_gvp.py -k "edge_embed" -x -q --timeout 120 --timeout-method thread > gpurun_out/t_embed.log 2>&1 || { tail -30 gpurun_out/t_embed.log; exit 3; }
tail -1 gpurun_out/t_embed.log
timeout -k 10 120 python scripts/mb_embed.py > gpurun_out/mb_embed.log 2>&1 || { tail gpurun_out/mb_embed.log; exit 1; }
grep K1e gpurun_out/mb_embed.log
bash scripts/gpu_round.sh || exit $?
bash scripts/gpu_profile.sh gvp 4 pmc > gpurun_out/prof_gvp.log 2>&1 || { tail gpurun_out/prof_gvp.log; exit 1; }
echo profile done
