#!/bin/bash
# Layer-3 expand conv (C = 256) on 64 x 128 streaming tiles (DLMPI_STREAM_C256_BN=128): test + A/B.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3_c256; mkdir -p $O
DLMPI_STREAM_C256_BN=128 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k stream1x1 -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; [ $rc -ne 0 ] && { grep -E "^FAILED|^ERROR|Error" $O/tests.log | head; exit 1; }
for i in 1 2; do
  for v in base bn128; do
    unset DLMPI_STREAM_C256_BN
    [ $v = bn128 ] && export DLMPI_STREAM_C256_BN=128
    for c in resnet50 resnet152; do
      timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 > $O/${c}_${v}_$i.log 2>&1 || { echo "bench $v failed"; exit 1; }
      echo "$c $v #$i $(grep -o '"value": [0-9.]*' $O/${c}_${v}_$i.log)"
    done
  done
done
