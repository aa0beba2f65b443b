#!/bin/bash
# Conv forward variant A/B (benchmarks/conv_ab.py) on ResNet-50 and UNet shapes.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python benchmarks/conv_ab.py --net unet512 ${AB_ARGS} > gpurun_out/ab_unet.log 2>&1 || { echo "unet rc=$?"; exit 1; }
timeout -k 10 300 python benchmarks/conv_ab.py --net resnet50 ${AB_ARGS} > gpurun_out/ab_r50.log 2>&1 || { echo "r50 rc=$?"; exit 1; }
echo ok
