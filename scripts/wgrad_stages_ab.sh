#!/bin/bash
# per-shape weight-gradient time, single- vs double-buffered, on the heaviest ResNet-50 wgrad shapes
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; export HSA_ENABLE_IPC_MODE_LEGACY=0
for v in 1 2; do
  for spec in "256,56,56,64,64,3,1,1" "256,14,14,256,256,3,1,1" "256,7,7,512,2048,1,1,0" "256,56,56,64,256,1,1,0" "256,28,28,128,128,3,1,1" "256,14,14,256,1024,1,1,0"; do
    r=$(DLMPI_WGRAD_STAGES=$v timeout -k 10 60 python benchmarks/conv_one.py --shape $spec --pass wgrad --iters 30 2>/dev/null | tail -1) || { echo "fail"; exit 1; }
    echo "stages=$v | $r"
  done
done
