#!/bin/bash
# Kernel-trace profiles: ResNet-50 with / without deferred weight-gradient reductions, ResNet-18
# CIFAR (eager), UNet-512 / UNet-1024.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
TAG=defer CONFIGS=resnet50 bash scripts/r4_prof.sh || exit 1
TAG=nodefer ARGS="--pin defer=0" CONFIGS=resnet50 bash scripts/r4_prof.sh || exit 1
TAG=cifar ARGS="--graph 0" CONFIGS=resnet18_cifar bash scripts/r4_prof.sh || exit 1
TAG=unet CONFIGS="unet512 unet1024" STEPS=3 bash scripts/r4_prof.sh || exit 1
