#!/bin/bash
# A/B of the K-loop structure (stages 1 vs 2) of the conv + wgrad kernels on ResNet-50 and UNet shapes.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
ONLY=${ONLY:-wgrad}
for st in 2 1; do
  DLMPI_CONV_STAGES=$st DLMPI_WGRAD_STAGES=$st timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -x -k "conv or linear or convT or unet" > gpurun_out/kernels_s$st.log 2>&1; echo "kernels s$st rc=$?"
  timeout -k 10 400 python benchmarks/conv_bench.py --stages $st --no_miopen --iters 10 --only $ONLY > gpurun_out/cb_r50_s$st.log 2>&1 || exit 1
  timeout -k 10 400 python benchmarks/conv_bench.py --net unet512 --stages $st --iters 10 --no_miopen --only $ONLY > gpurun_out/cb_unet_s$st.log 2>&1 || exit 1
done
