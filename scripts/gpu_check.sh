set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
python -c "import torch;print(torch.cuda.get_device_name(0), torch.version.hip)" > gpurun_out/env.log 2>&1
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/bench.log 2>&1
