#!/bin/bash
# Round-4 end-of-session validation: GPU tests, smoke, headline benches (all configs), and kernel-trace
# profiles of ResNet-50, UNet-512, UNet-1024 and ResNet-18 CIFAR (eager) for the profiles/ tables.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
NOLAB=1 CONFIGS="resnet50 resnet152 resnet18_cifar unet512 unet1024" TAG=final bash scripts/r4_check.sh || exit 1
TAG=final CONFIGS="resnet50 unet512 unet1024" STEPS=3 bash scripts/r4_prof.sh || exit 1
TAG=final_cifar ARGS="--graph 0" CONFIGS=resnet18_cifar bash scripts/r4_prof.sh || exit 1
