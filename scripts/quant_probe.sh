#!/bin/bash
# wave-quantization probe: time per image at batch sizes around the 1- and 2-wave boundaries
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; export HSA_ENABLE_IPC_MODE_LEGACY=0
for spec in "14,14,256,256,3,1,1 fwd" "14,14,1024,256,1,1,0 fwd" "28,28,128,128,3,1,1 fwd" "28,28,512,128,1,1,0 fwd" "14,14,256,1024,1,1,0 dgrad"; do
  set -- $spec
  for n in 192 240 248 256 264 320; do
    r=$(timeout -k 10 60 python benchmarks/conv_one.py --shape $n,$1 --pass $2 --iters 30 2>/dev/null | tail -1) || { echo fail; exit 1; }
    echo "N=$n | $r"
  done
done
