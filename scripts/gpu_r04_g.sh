#!/bin/bash
# fused-forward layer test, then the GVP (C3) bench line and its kernel-trace profile + HBM passes
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD/geometric-message-passing_amd
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_equivariant.py -k fused_forward > gpurun_out/pytest_fusedlayer.log 2>&1 || { cat gpurun_out/pytest_fusedlayer.log; exit 1; }
tail -2 gpurun_out/pytest_fusedlayer.log
timeout -k 10 300 python -u bench.py --workload gvp --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_gvp.log 2>&1 || exit 1
tail -c 1500 gpurun_out/bench_gvp.log
bash scripts/gpu_profile.sh gvp 5 pmc
