#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python benchmarks/conv_bench.py --iters 10 --no_miopen > gpurun_out/sp_r50_0.log 2>&1 || exit 1
timeout -k 10 400 python benchmarks/conv_bench.py --net unet512 --iters 10 --no_miopen --only fwd > gpurun_out/sp_u_0.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/sp_bench_0.log 2>&1 || exit 1
touch deeplearning_mpi_amd/csrc/kernels/conv_igemm.hip
DLMPI_HIPCC_FLAGS=-DDLMPI_SETPRIO=1 timeout -k 10 900 python -m deeplearning_mpi_amd.build > gpurun_out/sp_build.log 2>&1 || exit 1
timeout -k 10 400 python benchmarks/conv_bench.py --iters 10 --no_miopen > gpurun_out/sp_r50_1.log 2>&1 || exit 1
timeout -k 10 400 python benchmarks/conv_bench.py --net unet512 --iters 10 --no_miopen --only fwd > gpurun_out/sp_u_1.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/sp_bench_1.log 2>&1 || exit 1
