#!/bin/bash
# Producer BN-apply fused into the consumer conv1 (pro 3): tests, then ResNet-50 / ResNet-152 A/B.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3_fuse; mkdir -p $O
timeout -k 10 400 python -u -m pytest -q --timeout 180 --timeout-method thread tests/test_fuse_apply_gpu.py tests/test_models_gpu.py > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -ne 0 ] && { grep -E "^FAILED|^E  " $O/tests.log | head -20; exit 1; }
CONFIGS="resnet50 resnet152" STEPS=20 REPS=2 VARIANTS='base f0=DLMPI_FUSE_APPLY=0' bash scripts/env_ab3.sh
