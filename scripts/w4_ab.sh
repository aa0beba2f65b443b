#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python benchmarks/conv_bench.py --iters 10 --no_miopen > gpurun_out/w_r50_3.log 2>&1 || exit 1
timeout -k 10 400 python benchmarks/conv_bench.py --net unet512 --iters 10 --no_miopen > gpurun_out/w_u_3.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/w_bench_3.log 2>&1 || exit 1
touch deeplearning_mpi_amd/csrc/kernels/conv_igemm.hip
DLMPI_HIPCC_FLAGS=-DDLMPI_W128=4 timeout -k 10 900 python -m deeplearning_mpi_amd.build > gpurun_out/w_build.log 2>&1 || exit 1
timeout -k 10 400 python -m pytest tests/test_kernels_gpu.py -q -x -k conv > gpurun_out/w_kernels.log 2>&1; echo "kernels rc=$?"
timeout -k 10 400 python benchmarks/conv_bench.py --iters 10 --no_miopen > gpurun_out/w_r50_4.log 2>&1 || exit 1
timeout -k 10 400 python benchmarks/conv_bench.py --net unet512 --iters 10 --no_miopen > gpurun_out/w_u_4.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/w_bench_4.log 2>&1 || exit 1
