#!/bin/bash
# A/B of two builds of the package on the same box: ab_old/ (a saved copy) vs the working tree,
# conv forward default tiles (benchmarks/conv_ab.py), then full training steps of the working tree.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/bab
export HSA_ENABLE_IPC_MODE_LEGACY=0
for i in 1 2; do
  for v in old new; do
    for net in resnet50 unet512; do
      if [ $v = old ]; then export DLMPI_AB_ROOT=ab_old; else unset DLMPI_AB_ROOT; fi
      timeout -k 10 300 python benchmarks/conv_ab.py --net $net --variants default > gpurun_out/bab/${net}_${v}_$i.log 2>&1 || { echo "$net $v rc=$?"; exit 1; }
      echo "$net $v #$i $(tail -1 gpurun_out/bab/${net}_${v}_$i.log)"
    done
  done
done
