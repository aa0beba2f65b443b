#!/bin/bash
# Round-4 GPU call: the GPU tests, smoke, the headline benches and the per-shape conv table
# (production dispatch vs MIOpen).
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4_convtab; mkdir -p $O
NOLAB=1 CONFIGS="${CONFIGS:-resnet50 unet512 unet1024}" bash scripts/r4_check.sh || exit 1
cd $R && timeout -k 10 400 python benchmarks/conv_bench.py --net resnet50 --iters 20 > $O/conv_bench_r50.log 2>&1 || { echo convtab failed; tail -5 $O/conv_bench_r50.log; exit 1; }
echo convtab done
