#!/bin/bash
# A/B of the 256x128 conv tile threshold on ResNet-50 / UNet shapes (fwd + dgrad).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -m pytest tests/test_kernels_gpu.py -q -x > gpurun_out/kernels.log 2>&1; echo "kernels rc=$?"
for th in 1000000 1024 512; do
  timeout -k 10 400 python benchmarks/conv_bench.py --bm256_min_tiles $th --no_miopen --iters 10 --only fwd > gpurun_out/cb_r50_fwd_t$th.log 2>&1 || exit 1
  timeout -k 10 400 python benchmarks/conv_bench.py --bm256_min_tiles $th --no_miopen --iters 10 --only dgrad > gpurun_out/cb_r50_dgrad_t$th.log 2>&1 || exit 1
  timeout -k 10 400 python benchmarks/conv_bench.py --net unet512 --bm256_min_tiles $th --iters 10 --no_miopen --only fwd > gpurun_out/cb_unet_fwd_t$th.log 2>&1 || exit 1
done
