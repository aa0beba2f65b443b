#!/bin/bash
# Targeted GPU tests: ${TESTS} (pytest node ids / files), optional -k expression ${K}, one process.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && export HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out/gpu_tests${TAG:+_$TAG}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -m gpu -q -x --timeout 180 --timeout-method thread ${K:+-k "$K"} ${TESTS} > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log
if [ $rc -ne 0 ]; then grep -E "^FAILED|^ERROR|Error" $O/tests.log | head -20; exit 1; fi
exit 0
