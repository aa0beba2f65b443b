#!/bin/bash
# Round-6 wgrad3 check: the weight-gradient GPU tests, then same-box A/B of this tree vs abh.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && export HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out/r6_w3check; mkdir -p $O
timeout -k 10 400 python -u -m pytest -m gpu -q -x --timeout 180 --timeout-method thread -k "wgrad or benchscale or unet or graph" tests > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log
if [ $rc -ne 0 ]; then grep -E "^FAILED|^ERROR|Error" $O/tests.log | head -20; exit 1; fi
DIRS="abh ." CONFIGS="${CONFIGS:-unet512 resnet50 unet1024}" REPS=${REPS:-2} OUT=gpurun_out/r6_w3check/ab bash scripts/ab_rev.sh
