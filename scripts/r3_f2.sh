#!/bin/bash
# Fused producer BN-apply for consumers with several output tile columns (layer-3 conv1): tests + A/B.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3_f2; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_fuse_apply_gpu.py tests/test_kernels_gpu.py -k "fuse or apply or prologue or deferred" -x -q --timeout 180 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -ne 0 ] && { grep -E "^FAILED|^ERROR|Error" $O/tests.log | head -20; exit 1; }
for i in 1 2; do
  for v in base k128; do
    unset DLMPI_FUSE_APPLY_MAXK
    [ $v = k128 ] && export DLMPI_FUSE_APPLY_MAXK=128
    for c in resnet50 resnet152; do
      timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 > $O/${c}_${v}_$i.log 2>&1 || { echo "bench $c $v failed"; tail -5 $O/${c}_${v}_$i.log; exit 1; }
      echo "$c $v #$i $(grep -o '"value": [0-9.]*' $O/${c}_${v}_$i.log)"
    done
  done
done
