#!/bin/bash
# The reference's own workload at its precision: ResNet-18 CIFAR bs 128 in fp32 on
# the native kernels and in stock PyTorch fp32, plus both in bf16, on one box.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && export HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out/r6_fp32; mkdir -p $O
for p in fp32 bf16; do
  timeout -k 10 300 python bench.py --config resnet18_cifar --precision $p > $O/ours_$p.log 2>&1 || { echo "ours $p failed"; tail -5 $O/ours_$p.log; exit 1; }
  echo "ours $p $(grep -o '"value": [0-9.]*' $O/ours_$p.log) $(grep -o '"hipgraph": [a-z]*' $O/ours_$p.log)"
  timeout -k 10 400 python benchmarks/torch_baseline.py --config resnet18_cifar --precision $p --steps 50 --warmup 10 > $O/stock_$p.log 2>&1 || { echo "stock $p failed"; tail -5 $O/stock_$p.log; exit 1; }
  echo "stock $p $(grep -o '"value": [0-9.]*' $O/stock_$p.log)"
done
exit 0
