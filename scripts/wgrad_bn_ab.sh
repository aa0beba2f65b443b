#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
DLMPI_WGRAD_BN=256 timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -x -k "wgrad or linear or convT or unet" > gpurun_out/kernels_bn256.log 2>&1; echo "kernels rc=$?"
for bn in 128 256; do
  DLMPI_WGRAD_BN=$bn timeout -k 10 400 python benchmarks/conv_bench.py --iters 10 --no_miopen --only wgrad > gpurun_out/cb_wg_bn$bn.log 2>&1 || exit 1
  DLMPI_WGRAD_BN=$bn timeout -k 10 400 python benchmarks/conv_bench.py --net unet512 --iters 10 --no_miopen --only wgrad > gpurun_out/cb_wgu_bn$bn.log 2>&1 || exit 1
done
