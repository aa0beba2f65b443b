#!/bin/bash
# GPU validation: full GPU test suite (hang-safe), smoke, headline bench.  Output: gpurun_out/$1/
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/${1:-r2_check}
cd "$R" && mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 180 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?
grep -E "passed|failed|error" $O/gpu_tests.log | tail -3
[ $rc -eq 0 ] || { grep -E "FAILED|Error|error" $O/gpu_tests.log | head -20; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || exit 1
cat $O/bench.log | grep metric
