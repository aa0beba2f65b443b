#!/bin/bash
# A/B of conv kernel knobs on the output-heavy 1x1 (expand) shapes and a reduce-layer dgrad
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/expand_ab; mkdir -p $O
for v in "X=0" "DLMPI_NT_STORE=1" "DLMPI_CONV_BM=64" "DLMPI_CONV_BM=256" "DLMPI_CONV_STAGES=2"; do
  for spec in "256,56,56,64,256,1,1,0 fwd" "256,28,28,128,512,1,1,0 fwd" "256,14,14,256,1024,1,1,0 fwd" "256,56,56,256,64,1,1,0 dgrad" "256,14,14,256,256,3,1,1 fwd"; do
    set -- $spec
    r=$(env $v timeout -k 10 60 python benchmarks/conv_one.py --shape $1 --pass $2 --iters 30 2>/dev/null | tail -1) || { echo "fail $v $spec"; exit 1; }
    echo "$v | $r"
  done
done
