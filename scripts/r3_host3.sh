#!/bin/bash
# Host issue time after the cheaper side-stream switch + arena check (A/B needs no knob: compare with
# profiles/r3_host), and the benches.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3_host3; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_ddp_rccl_gpu.py tests/test_comm_ordering_gpu.py -x -q --timeout 180 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; [ $rc -ne 0 ] && { grep -E "^FAILED|^ERROR|Error" $O/tests.log | head -20; exit 1; }
for c in resnet152 resnet50; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 --rccl1 1 --host_time 10 --pyprof 5 > $O/pyprof_$c.log 2>&1 || { echo "pyprof $c failed"; tail -5 $O/pyprof_$c.log; exit 1; }
  echo "$c $(grep -o '"value": [0-9.]*' $O/pyprof_$c.log) $(grep -o 'host_issue_ms_per_step_median": [0-9.]*' $O/pyprof_$c.log | head -1) $(grep -o '"host_over_gpu": [0-9.]*' $O/pyprof_$c.log | head -1)"
done
