#!/bin/bash
# Re-check of HEAD after the 256-row 1x1 tile change: full GPU suite, smoke, headline bench, the --rccl1 path
# world-1 RCCL communicator, streaming-dgrad grid sized for the channels).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3_final3; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 180 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log
if [ $rc -ne 0 ]; then grep -E "^FAILED|^ERROR" $O/tests.log | head -30; [ $rc -ge 124 ] && exit 1; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { echo bench failed; exit 1; }
echo "bench $(grep -o '"value": [0-9.]*' $O/bench.log)"
timeout -k 10 300 python bench.py --rccl1 1 --steps 20 --warmup 5 > $O/bench_rccl1.log 2>&1 || { echo rccl1 failed; tail -5 $O/bench_rccl1.log; exit 1; }
echo "rccl1 $(grep -o '"value": [0-9.]*' $O/bench_rccl1.log) $(grep -o '"dgrad_stream_blocks": [0-9]*' $O/bench_rccl1.log) $(grep -o '"rccl_channels": "[0-9]*"' $O/bench_rccl1.log)"
