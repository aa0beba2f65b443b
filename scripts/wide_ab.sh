#!/bin/bash
# 128x256 wide tile vs default on the short-reduction wide-output shapes (conv_one), then bench
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; export HSA_ENABLE_IPC_MODE_LEGACY=0
for v in 0 256; do
  for spec in "256,56,56,64,256,1,1,0 fwd" "256,28,28,128,512,1,1,0 fwd" "256,14,14,256,1024,1,1,0 fwd" "256,56,56,256,64,1,1,0 dgrad" "256,28,28,512,128,1,1,0 dgrad" "256,14,14,1024,256,1,1,0 dgrad" "256,56,56,64,64,1,1,0 fwd"; do
    set -- $spec
    r=$(DLMPI_CONV_WIDE=$v timeout -k 10 60 python benchmarks/conv_one.py --shape $1 --pass $2 --iters 30 2>/dev/null | tail -1) || { echo "fail $v $spec"; exit 1; }
    echo "wide=$v | $r"
  done
done
AB_SETS="DLMPI_CONV_WIDE=0;DLMPI_CONV_WIDE=256" AB_REPS=2 bash scripts/multi_ab.sh
