#!/bin/bash
# General weight-gradient grid target (DLMPI_WGRAD_BLOCKS, default 512) re-measured after the
# round-3 changes: fewer splits = smaller fp32 slabs for the two reduction kernels + CUs left to the
# data-gradient chain.  Then the current ResNet-50 kernel profile.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && export HSA_ENABLE_IPC_MODE_LEGACY=0
CONFIGS="resnet50 resnet152 unet512" STEPS=10 REPS=2 VARIANTS='base b256=DLMPI_WGRAD_BLOCKS=256 b384=DLMPI_WGRAD_BLOCKS=384 b768=DLMPI_WGRAD_BLOCKS=768' bash scripts/env_ab3.sh || exit 1
O=gpurun_out/r3_prof2; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$O/prof_resnet50" -o r -- python3 "$R/bench.py" --steps 5 --warmup 2 > "$R/$O/prof_resnet50.log" 2>&1 || { echo "prof failed"; exit 1; }
echo "prof done $(grep -o '"value": [0-9.]*' $R/$O/prof_resnet50.log)"
