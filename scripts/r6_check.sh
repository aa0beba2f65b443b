#!/bin/bash
# Round-6 check of the working tree: the GPU suite, smoke, the world-1 collective benchmark, and the
# headline bench plain and through a world-1 RCCL reducer with the per-bucket probe.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && export HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out/r6_check${TAG:+_$TAG}; mkdir -p $O
if [ -z "$NOTEST" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 180 --timeout-method thread ${TESTS} > $O/tests.log 2>&1
  rc=$?; tail -1 $O/tests.log
  if [ $rc -ne 0 ]; then grep -E "^FAILED|^ERROR|Error" $O/tests.log | head -20; exit 1; fi
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail -5 $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log
fi
timeout -k 10 300 python benchmarks/comm_bench.py --gpus 1 > $O/comm_bench_w1.jsonl 2> $O/comm_bench_w1.err || { echo comm_bench failed; tail -5 $O/comm_bench_w1.err; exit 1; }
tail -1 $O/comm_bench_w1.jsonl | cut -c1-300
for c in ${CONFIGS:-resnet50}; do
  timeout -k 10 300 python bench.py --config $c > $O/bench_$c.log 2>&1 || { echo "bench $c failed"; tail -5 $O/bench_$c.log; exit 1; }
  echo "bench $c $(grep -o '"value": [0-9.]*' $O/bench_$c.log) $(grep -o '"ms_per_step": [0-9.]*' $O/bench_$c.log)"
done
timeout -k 10 300 python bench.py --config resnet50 --rccl1 1 > $O/bench_resnet50_rccl1.log 2>&1 || { echo "rccl1 failed"; tail -5 $O/bench_resnet50_rccl1.log; exit 1; }
echo "bench resnet50 rccl1 $(grep -o '"value": [0-9.]*' $O/bench_resnet50_rccl1.log) $(grep -o '"comm_tail_ms": [-0-9.]*' $O/bench_resnet50_rccl1.log)"
exit 0
