#!/bin/bash
# Full GPU suite (no -x), then the wgrad PMC probes.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3_check; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 180 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log
if [ $rc -ne 0 ]; then grep -E "^FAILED|^ERROR" $O/tests.log | head -30; [ $rc -ge 124 ] && exit 1; fi
bash scripts/r3_pmc_wgrad.sh
