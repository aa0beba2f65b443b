#!/bin/bash
# bn2 apply rebuilt in the streaming conv3's prologue (engine.STREAM_PRO): tests + A/B.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3_spro; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_stream_pro_gpu.py tests/test_kernels_gpu.py -k "stream or pro or deferred" -x -q --timeout 180 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -ne 0 ] && { grep -E "^FAILED|^ERROR|Error|assert" $O/tests.log | head -20; exit 1; }
for i in 1 2; do
  for v in base p0; do
    unset DLMPI_STREAM_PRO_FWD
    [ $v = p0 ] && export DLMPI_STREAM_PRO_FWD=0
    for c in resnet50 resnet152; do
      timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 > $O/${c}_${v}_$i.log 2>&1 || { echo "bench $c $v failed"; tail -5 $O/${c}_${v}_$i.log; exit 1; }
      echo "$c $v #$i $(grep -o '"value": [0-9.]*' $O/${c}_${v}_$i.log)"
    done
  done
done
