#!/bin/bash
# Host-side profile of the eager ResNet-152 / ResNet-50 step (--pyprof) with a live reducer on a
# world-1 RCCL communicator, plus current UNet / CIFAR numbers.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3_host; mkdir -p $O
for c in resnet152 resnet50; do
  timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 3 --rccl1 1 --host_time 10 --pyprof 5 > $O/pyprof_$c.log 2>&1 || { echo "pyprof $c failed"; tail -5 $O/pyprof_$c.log; exit 1; }
  echo "$c $(grep -o '"host_over_gpu": [0-9.]*' $O/pyprof_$c.log | head -1)"
done
for c in unet512 resnet18_cifar; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 > $O/bench_$c.log 2>&1 || { echo "bench $c failed"; exit 1; }
  echo "$c $(grep -o '"value": [0-9.]*' $O/bench_$c.log)"
done
