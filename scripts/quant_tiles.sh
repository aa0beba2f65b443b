#!/bin/bash
# tile choice on the wave-quantized ResNet-50 shapes (bs 256)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; export HSA_ENABLE_IPC_MODE_LEGACY=0
for v in "X=0" "DLMPI_CONV_BM=64" "DLMPI_CONV_BM=256"; do
  for spec in "256,14,14,1024,256,1,1,0 fwd" "256,14,14,256,1024,1,1,0 dgrad" "256,28,28,512,128,1,1,0 fwd" "256,28,28,128,128,3,1,1 fwd" "256,28,28,128,128,3,1,1 dgrad" "256,7,7,512,2048,1,1,0 fwd" "256,7,7,2048,512,1,1,0 dgrad" "256,14,14,256,256,3,1,1 dgrad"; do
    set -- $spec
    r=$(env $v timeout -k 10 60 python benchmarks/conv_one.py --shape $1 --pass $2 --iters 30 2>/dev/null | tail -1) || { echo fail; exit 1; }
    echo "$v | $r"
  done
done
