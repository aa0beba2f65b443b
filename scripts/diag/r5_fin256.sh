#!/bin/bash
# 256-thread wave-local finalize: BN tests, then same-box A/B against the HEAD tree (abh) on ResNet-50 / CIFAR.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && export HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out/r5_fin256; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_fuse_apply_gpu.py tests/test_dual_dgrad_gpu.py > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit 1
OUT=gpurun_out/r5_fin256/ab DIRS="abh ." CONFIGS="${CONFIGS:-resnet50 resnet18_cifar}" REPS=${REPS:-3} STEPS=30 bash scripts/ab_rev.sh
