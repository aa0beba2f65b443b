#!/bin/bash
# End-of-session bench of every BASELINE config on HEAD (one box).  Output: gpurun_out/r3_allcfg/
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && export HSA_ENABLE_IPC_MODE_LEGACY=0
O="$R/gpurun_out/r3_allcfg"; mkdir -p "$O"
for c in resnet50 resnet152 unet512 unet1024 resnet18_cifar; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 > "$O/$c.log" 2>&1 || { echo "bench $c failed"; tail -5 "$O/$c.log"; exit 1; }
  echo "$c $(grep -o '"value": [0-9.]*' $O/$c.log) $(grep -o '"vs_baseline": [0-9.]*' $O/$c.log)"
done
