#!/bin/bash
# First GPU pass: kernel numerics, model numerics, smoke, short bench + stock baseline.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
python -c "import torch; print(torch.cuda.get_device_name(0))" > gpurun_out/dev.txt 2>&1
timeout -k 10 900 python -m pytest tests/test_kernels_gpu.py -x -q -m gpu > gpurun_out/kernels.log 2>&1; echo "kernels rc=$?"
