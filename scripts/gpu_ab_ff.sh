# A/B of the GVP step with K17 (the fused node feed-forward) on and off, alternating runs.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/ab_ff
mkdir -p $D
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_gvp.py -k "ff" > $D/tests.log 2>&1 || { tail -20 $D/tests.log; exit 1; }
tail -1 $D/tests.log
for k in 1 2; do
  for ff in 1 0; do
    GMP_AB_FF=$ff timeout -k 10 300 python3 scripts/ab_ff_bench.py > $D/b.json 2> $D/b.err || { tail -5 $D/b.err; exit 1; }
    echo "ff=$ff $(cat $D/b.json)"
  done
done
