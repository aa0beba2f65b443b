#!/bin/bash
# Round-3 refresh of the per-shape ResNet-50 conv table (ours vs MIOpen), same harness as
# scripts/r2_diag.sh's first step.  Output: gpurun_out/r3_convtab/
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && export HSA_ENABLE_IPC_MODE_LEGACY=0
O="$R/gpurun_out/r3_convtab"; mkdir -p "$O"
timeout -k 10 400 python -u benchmarks/conv_bench.py --net resnet50 --iters 20 > "$O/conv_bench_r50.log" 2>&1 || { echo "conv_bench failed"; tail -5 "$O/conv_bench_r50.log"; exit 1; }
tail -1 "$O/conv_bench_r50.log"
