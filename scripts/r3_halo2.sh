#!/bin/bash
# halo tiles restricted to >= 28^2 grids without a 256x256 plan: tests + bench A/B incl. UNet-1024
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3_halo2; mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --timeout 180 --timeout-method thread tests/test_kernels_gpu.py -k "halo or conv" > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -ne 0 ] && { grep -E "^FAILED|^E  " $O/tests.log | head -20; exit 1; }
CONFIGS="resnet50 unet512 unet1024" STEPS=8 REPS=2 VARIANTS='base h0=DLMPI_CONV_HALO=0' bash scripts/env_ab3.sh
