#!/bin/bash
# GPU tests + A/B of the channel-fixed BN apply kernels (DLMPI_EW_ROWS) on full training steps.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/tests.log; exit 1; }
for i in 1 2; do
  for v in 0 1; do
    DLMPI_EW_ROWS=$v timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/ew_r50_${v}_$i.log 2>&1 || exit 1
  done
done
for v in 0 1; do
  DLMPI_EW_ROWS=$v timeout -k 10 300 python bench.py --config unet512 --steps 8 --warmup 3 > gpurun_out/ew_unet_${v}.log 2>&1 || exit 1
done
grep -h -o '"value": [0-9.]*' gpurun_out/ew_*.log
