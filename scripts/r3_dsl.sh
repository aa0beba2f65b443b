#!/bin/bash
# Downsample branch after the fused conv1 (resnet._DS_AFTER_CONV1) A/B + model GPU tests.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3_dsl; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_fuse_apply_gpu.py tests/test_models_gpu.py tests/test_dual_dgrad_gpu.py -x -q --timeout 180 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -ne 0 ] && { grep -E "^FAILED|^ERROR|Error" $O/tests.log | head -20; exit 1; }
for i in 1 2; do
  for v in base l0; do
    unset DLMPI_DS_AFTER_CONV1
    [ $v = l0 ] && export DLMPI_DS_AFTER_CONV1=0
    for c in resnet50 resnet152; do
      timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 > $O/${c}_${v}_$i.log 2>&1 || { echo "bench $c $v failed"; tail -5 $O/${c}_${v}_$i.log; exit 1; }
      echo "$c $v #$i $(grep -o '"value": [0-9.]*' $O/${c}_${v}_$i.log)"
    done
  done
done
