#!/bin/bash
# A/B of the conv kernel's K-loop structure (DLMPI_CONV_STAGES 1 vs 2) on ResNet-50 and UNet shapes.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -m pytest tests/test_kernels_gpu.py -q -x > gpurun_out/kernels.log 2>&1; echo "kernels rc=$?"
for st in 2 1; do
  DLMPI_CONV_STAGES=$st timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -x -k "conv" > gpurun_out/kernels_s$st.log 2>&1; echo "kernels s$st rc=$?"
  timeout -k 10 400 python benchmarks/conv_bench.py --stages $st --no_miopen --iters 10 > gpurun_out/cb_r50_s$st.log 2>&1 || exit 1
  timeout -k 10 400 python benchmarks/conv_bench.py --net unet512 --stages $st --iters 10 --no_miopen > gpurun_out/cb_unet_s$st.log 2>&1 || exit 1
done
