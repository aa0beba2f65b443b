#!/bin/bash
# A/B of the dual 1x1 data gradient variants on ResNet-50 (alternating on one box)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/dual_ab && export HSA_ENABLE_IPC_MODE_LEGACY=0
for i in 1 2; do
  for v in "DLMPI_DUAL_DGRAD=0" "DLMPI_DUAL_DGRAD=1" "DLMPI_DUAL_MIN_ROWS=802816" "DLMPI_DUAL_WGRAD_PRO=1" "DLMPI_DUAL_MIN_ROWS=802816 DLMPI_DUAL_WGRAD_PRO=1"; do
    tag=$(echo $v | tr ' =' '_-')
    env $v timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/dual_ab/${tag}_$i.log 2>&1 || { echo "bench $v rc=$?"; tail -20 gpurun_out/dual_ab/${tag}_$i.log; exit 1; }
    echo "$v #$i $(grep -o '"value": [0-9.]*' gpurun_out/dual_ab/${tag}_$i.log)"
  done
done
