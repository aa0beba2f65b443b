#!/bin/bash
# Streaming dgrad v2 (z2, in-place output staging): GPU tests, timings, bench A/B over grid sizes.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3_dgs2; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_dgrad_stream_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -ne 0 ] && { grep -E "^FAILED|^ERROR|Error" $O/tests.log | head -20; exit 1; }
timeout -k 10 300 python benchmarks/dgrad_stream_bench.py > $O/times.log 2>&1 || { tail $O/times.log; exit 1; }
cat $O/times.log
for i in 1 2; do
  for v in base b512 b1024 d0; do
    unset DLMPI_DGRAD_STREAM DLMPI_DGS_BLOCKS
    case $v in d0) export DLMPI_DGRAD_STREAM=0;; b512) export DLMPI_DGS_BLOCKS=512;; b1024) export DLMPI_DGS_BLOCKS=1024;; esac
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/resnet50_${v}_$i.log 2>&1 || { echo "bench $v failed"; tail -5 $O/resnet50_${v}_$i.log; exit 1; }
    echo "resnet50 $v #$i $(grep -o '"value": [0-9.]*' $O/resnet50_${v}_$i.log)"
  done
done
