#!/bin/bash
# Grid-size knobs re-tuned after the streaming data gradient (one persistent block per CU on the main
# stream): ResNet-50, 2 alternating reps per variant.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3_sweep; mkdir -p $O
for i in 1 2; do
  for v in base wg256 wg1024 dgs224 dgs192 w3b256; do
    unset DLMPI_WGRAD_BLOCKS DLMPI_DGS_BLOCKS DLMPI_WGRAD3_BLOCKS
    case $v in
      wg256) export DLMPI_WGRAD_BLOCKS=256;; wg1024) export DLMPI_WGRAD_BLOCKS=1024;;
      dgs224) export DLMPI_DGS_BLOCKS=224;; dgs192) export DLMPI_DGS_BLOCKS=192;;
      w3b256) export DLMPI_WGRAD3_BLOCKS=256;;
    esac
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/resnet50_${v}_$i.log 2>&1 || { echo "bench $v failed"; tail -5 $O/resnet50_${v}_$i.log; exit 1; }
    echo "resnet50 $v #$i $(grep -o '"value": [0-9.]*' $O/resnet50_${v}_$i.log)"
  done
done
