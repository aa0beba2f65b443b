#!/bin/bash
# More repetitions: CIFAR eager/graph old (ab_s3) vs new; ResNet-50 / ResNet-152 new default vs the
# old dual threshold (DLMPI_DUAL_MIN_ROWS=200704).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && export HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out/r3_cifar_ab3; mkdir -p $O
for i in 1 2 3; do
  for v in old new; do
    d=$R; [ $v = old ] && d=$R/ab_s3
    (cd $d && timeout -k 10 300 python bench.py --config resnet18_cifar --steps 100 --warmup 5 > $O/cifar_eager_${v}_$i.log 2>&1) || { echo "cifar eager $v failed"; exit 1; }
    (cd $d && timeout -k 10 300 python bench.py --config resnet18_cifar --graph 1 --steps 100 --warmup 5 > $O/cifar_graph_${v}_$i.log 2>&1) || { echo "cifar $v failed"; exit 1; }
    echo "cifar $v #$i eager $(grep -o '"value": [0-9.]*' $O/cifar_eager_${v}_$i.log) graph $(grep -o '"value": [0-9.]*' $O/cifar_graph_${v}_$i.log)"
  done
done
for i in 1 2; do
  for v in base d200k; do
    unset DLMPI_DUAL_MIN_ROWS
    [ $v = d200k ] && export DLMPI_DUAL_MIN_ROWS=200704
    for c in resnet50 resnet152; do
      timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 > $O/${c}_${v}_$i.log 2>&1 || { echo "bench $v failed"; exit 1; }
      echo "$c $v #$i $(grep -o '"value": [0-9.]*' $O/${c}_${v}_$i.log)"
    done
  done
done
