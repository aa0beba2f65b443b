#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
DLMPI_CONV_STAGES=3 timeout -k 10 400 python -m pytest tests/test_kernels_gpu.py -q -x -k "conv" > gpurun_out/kernels_s3.log 2>&1; echo "kernels s3 rc=$?"
for st in 1 3; do
  DLMPI_CONV_STAGES=$st timeout -k 10 400 python benchmarks/conv_bench.py --iters 10 --no_miopen > gpurun_out/s3_r50_$st.log 2>&1 || exit 1
  DLMPI_CONV_STAGES=$st timeout -k 10 400 python benchmarks/conv_bench.py --net unet512 --iters 10 --no_miopen > gpurun_out/s3_u_$st.log 2>&1 || exit 1
done
