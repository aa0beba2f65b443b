#!/bin/bash
# Session-3 baseline on a fresh box: GPU suite, smoke, headline bench, host-issue probe + rocprof.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3_s3_base; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 180 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log
if [ $rc -ne 0 ]; then grep -E "^FAILED|^ERROR" $O/tests.log | head -30; [ $rc -ge 124 ] && exit 1; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; exit 1; }
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { echo bench failed; exit 1; }
tail -1 $O/bench.log
bash scripts/r3_prof.sh
