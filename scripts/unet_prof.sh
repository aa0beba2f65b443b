#!/bin/bash
# Kernel profile of the UNet 512^2 config (ours).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_unet" -o unet --output-format csv -- python "$R/bench.py" --config unet512 --steps 3 --warmup 2 > "$R/gpurun_out/prof_unet.log" 2>&1
echo "prof rc=$?"
