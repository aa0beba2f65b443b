#!/bin/bash
# Streaming 1x1 data gradient: GPU tests, per-shape timing, ResNet-50 bench A/B (alternating).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3_dgs; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_dgrad_stream_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -ne 0 ] && { grep -E "^FAILED|^ERROR|Error" $O/tests.log | head -20; exit 1; }
timeout -k 10 300 python benchmarks/dgrad_stream_bench.py > $O/times.log 2>&1 || { cat $O/times.log | tail; exit 1; }
cat $O/times.log
for i in 1 2; do
  for v in base d0; do
    if [ $v = d0 ]; then export DLMPI_DGRAD_STREAM=0; else unset DLMPI_DGRAD_STREAM; fi
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/resnet50_${v}_$i.log 2>&1 || { echo "bench $v failed"; tail -5 $O/resnet50_${v}_$i.log; exit 1; }
    echo "resnet50 $v #$i $(grep -o '"value": [0-9.]*' $O/resnet50_${v}_$i.log)"
  done
done
