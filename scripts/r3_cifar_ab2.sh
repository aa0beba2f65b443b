#!/bin/bash
# ResNet-18 CIFAR (the reference's own run) and ResNet-50: session-3 start tree (ab_s3/, abc1b8b) vs
# the working tree, same box, alternating; plus DLMPI_DUAL_MIN_ROWS=802816 (dual only at layer 1).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && export HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out/r3_cifar_ab2; mkdir -p $O
for i in 1 2; do
  for v in old new; do
    d=$R; [ $v = old ] && d=$R/ab_s3
    (cd $d && timeout -k 10 300 python bench.py --config resnet18_cifar --graph 1 --steps 100 --warmup 5 > $O/cifar_graph_${v}_$i.log 2>&1) || { echo "cifar $v failed"; tail -5 $O/cifar_graph_${v}_$i.log; exit 1; }
    (cd $d && timeout -k 10 300 python bench.py --config resnet18_cifar --steps 100 --warmup 5 > $O/cifar_eager_${v}_$i.log 2>&1) || { echo "cifar eager $v failed"; exit 1; }
    echo "cifar $v #$i graph $(grep -o '"value": [0-9.]*' $O/cifar_graph_${v}_$i.log) eager $(grep -o '"value": [0-9.]*' $O/cifar_eager_${v}_$i.log)"
  done
  for v in base dual1; do
    unset DLMPI_DUAL_MIN_ROWS
    [ $v = dual1 ] && export DLMPI_DUAL_MIN_ROWS=802816
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/resnet50_${v}_$i.log 2>&1 || { echo "bench $v failed"; exit 1; }
    echo "resnet50 $v #$i $(grep -o '"value": [0-9.]*' $O/resnet50_${v}_$i.log)"
  done
done
