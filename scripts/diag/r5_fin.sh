#!/bin/bash
# Finalize-prelude fusion: kernel tests, then same-box A/B (fusion on / off) on CIFAR and ResNet-50.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && export HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out/r5_fin; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_fin_fuse_gpu.py > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit 1
OUT=gpurun_out/r5_fin/ab VARIANTS="on off:--pin+fin_fuse=0" CONFIGS="resnet18_cifar resnet50" REPS=${REPS:-2} STEPS=30 bash scripts/ab.sh
