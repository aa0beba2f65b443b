#!/bin/bash
# Dual data gradient at layer 1 at all (threshold above every layer = off) vs the default.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3_dual_ab; mkdir -p $O
for i in 1 2; do
  for v in base off; do
    unset DLMPI_DUAL_MIN_ROWS
    [ $v = off ] && export DLMPI_DUAL_MIN_ROWS=100000000
    for c in resnet50 resnet152; do
      timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 > $O/${c}_${v}_$i.log 2>&1 || { echo "bench $c $v failed"; exit 1; }
      echo "$c $v #$i $(grep -o '"value": [0-9.]*' $O/${c}_${v}_$i.log)"
    done
  done
done
