#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for bm in 0 64 128; do
  for sh in "256,56,56,64,256,1,1,0" "256,56,56,256,64,1,1,0" "256,28,28,128,512,1,1,0" "256,14,14,256,256,3,1,1" "256,56,56,64,64,3,1,1"; do
    DLMPI_CONV_BM=$bm timeout -k 10 60 python benchmarks/conv_one.py --shape $sh --pass fwd --iters 20 >> gpurun_out/occ_bm$bm.log 2>&1 || exit 1
    DLMPI_CONV_BM=$bm timeout -k 10 60 python benchmarks/conv_one.py --shape $sh --pass dgrad --iters 20 >> gpurun_out/occ_bm$bm.log 2>&1 || exit 1
  done
done
