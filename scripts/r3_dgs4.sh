#!/bin/bash
# Streaming dgrad v4 (K = 512 with residual / mask bits on 32 x 64 tiles): tests, timings, ResNet A/B
# (base vs DLMPI_DGS_K512=0 equivalent: the general kernel for K = 512 via DLMPI_DGRAD_STREAM=0 is too
# coarse, so compare against the previous commit's behaviour with DLMPI_DGS_NO512=1).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3_dgs4; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_dgrad_stream_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -ne 0 ] && { grep -E "^FAILED|^ERROR|Error" $O/tests.log | head -20; exit 1; }
timeout -k 10 300 python benchmarks/dgrad_stream_bench.py > $O/times.log 2>&1 || { tail $O/times.log; exit 1; }
cat $O/times.log
for i in 1 2; do
  for v in base n512; do
    unset DLMPI_DGS_NO512
    [ $v = n512 ] && export DLMPI_DGS_NO512=1
    for c in resnet50 resnet152; do
      timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 > $O/${c}_${v}_$i.log 2>&1 || { echo "bench $c $v failed"; tail -5 $O/${c}_${v}_$i.log; exit 1; }
      echo "$c $v #$i $(grep -o '"value": [0-9.]*' $O/${c}_${v}_$i.log)"
    done
  done
done
