#!/bin/bash
# Full GPU validation + headline bench + UNet config + conv bench summaries.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -m pytest tests -q -m gpu -x > gpurun_out/allgpu.log 2>&1; echo "allgpu rc=$?"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; echo "smoke rc=$?"
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/bench.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --config unet512 --steps 10 --warmup 3 > gpurun_out/cfg_unet512_ours.log 2>&1 || exit 1
timeout -k 10 400 python benchmarks/conv_bench.py --net unet512 --iters 10 --no_miopen > gpurun_out/cb_unet.log 2>&1 || exit 1
timeout -k 10 400 python benchmarks/conv_bench.py --iters 10 --no_miopen > gpurun_out/cb_r50.log 2>&1 || exit 1
