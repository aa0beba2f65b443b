#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -m pytest tests/test_kernels_gpu.py -q -x > gpurun_out/kernels.log 2>&1; echo "kernels rc=$?"
timeout -k 10 400 python benchmarks/conv_bench.py --iters 10 --no_miopen --only wgrad > gpurun_out/cbr_wg.log 2>&1 || exit 1
timeout -k 10 400 python benchmarks/conv_bench.py --net unet512 --iters 10 --no_miopen --only wgrad > gpurun_out/cbu_wg.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/bench.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --config unet512 --steps 10 --warmup 3 > gpurun_out/cfg_unet512_ours.log 2>&1 || exit 1
