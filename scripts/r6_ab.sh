#!/bin/bash
# Targeted GPU tests (K) then a same-box A/B of this tree vs abh (CONFIGS, REPS).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && export HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out/r6_ab${TAG:+_$TAG}; mkdir -p $O
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest -m gpu -q -x --timeout 180 --timeout-method thread -k "$K" tests > $O/tests.log 2>&1
  rc=$?; tail -1 $O/tests.log
  if [ $rc -ne 0 ]; then grep -E "^FAILED|^ERROR|Error" $O/tests.log | head -20; exit 1; fi
fi
DIRS="abh ." CONFIGS="${CONFIGS:-resnet50}" REPS=${REPS:-2} OUT=gpurun_out/r6_ab${TAG:+_$TAG}/ab bash scripts/ab_rev.sh
