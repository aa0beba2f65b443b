#!/bin/bash
# GPU tests (${TESTS}), then same-box A/B of this tree against the HEAD worktree (abh) on ${CONFIGS}.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && export HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out/${TAG:-r5_ab}; mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TTLIM:-600} python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu $TESTS > $O/tests.log 2>&1
  rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit 1
fi
OUT=gpurun_out/${TAG:-r5_ab}/ab DIRS="abh ." CONFIGS="${CONFIGS:-resnet50}" REPS=${REPS:-3} STEPS=${STEPS:-30} bash scripts/ab_rev.sh
