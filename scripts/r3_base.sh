#!/bin/bash
# Round-3 session-start baseline on one box: headline bench, ResNet-18 CIFAR eager/graph repeats,
# kernel-trace of the CIFAR step (kernel counts per step) and of ResNet-50.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3_base; mkdir -p $O
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_r50_$i.log 2>&1 || { echo "bench rc=$?"; tail -5 $O/bench_r50_$i.log; exit 1; }
  echo "r50 $i $(grep -o '"value": [0-9.]*' $O/bench_r50_$i.log)"
done
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --config resnet18_cifar --steps 50 --warmup 5 > $O/cifar_eager_$i.log 2>&1 || exit 1
  echo "cifar eager $i $(grep -o '"value": [0-9.]*' $O/cifar_eager_$i.log)"
  timeout -k 10 300 python bench.py --config resnet18_cifar --graph 1 --steps 50 --warmup 5 > $O/cifar_graph_$i.log 2>&1 || exit 1
  echo "cifar graph $i $(grep -o '"value": [0-9.]*' $O/cifar_graph_$i.log)"
done
cd /tmp && export TMPDIR=/tmp
for c in resnet18_cifar resnet50; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$O/prof_$c" -o r -- python3 "$R/bench.py" --config $c --steps 5 --warmup 2 > "$R/$O/prof_$c.log" 2>&1 || { echo "prof $c failed"; exit 1; }
  echo "prof $c done"
done
