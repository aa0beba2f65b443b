#!/bin/bash
# Round-2 baseline on a fresh box: GPU test suite, smoke, headline bench, rocprofv3 kernel stats.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r2_base
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r2_base
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || exit 1
cat $O/bench.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$O/prof" -o r50 -- python3 "$R/bench.py" --steps 5 --warmup 2 > "$R/$O/prof.log" 2>&1 || exit 1
echo done
