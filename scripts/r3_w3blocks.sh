#!/bin/bash
# wgrad3 grid size / tile A/B on the two configs where it runs beside the data-gradient chain
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && export HSA_ENABLE_IPC_MODE_LEGACY=0
CONFIGS="resnet50 unet512" STEPS=10 REPS=2 VARIANTS='base b160=DLMPI_WGRAD3_BLOCKS=160 b96=DLMPI_WGRAD3_BLOCKS=96 kt64=DLMPI_WGRAD3_KT=64 kt64b160=DLMPI_WGRAD3_KT=64,DLMPI_WGRAD3_BLOCKS=160 w0=DLMPI_WGRAD3=0' bash scripts/env_ab3.sh
