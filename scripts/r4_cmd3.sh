#!/bin/bash
# Round-4: targeted GPU tests, then same-box A/B of the deferred weight-gradient reductions and of
# round 3 vs HEAD on the CIFAR config, then kernel-trace profiles of CIFAR (HEAD and round 3).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
K='wgrad_reduce_batched or deferred or pipelined' TESTS='tests/test_wgrad_defer_gpu.py tests/test_kernels_gpu.py' bash scripts/r4_t.sh || exit 1
VARIANTS='base nodefer:--pin+defer=0' CONFIGS='resnet50' REPS=2 bash scripts/ab.sh || exit 1
VARIANTS='base nodefer:--pin+defer=0 w3b160:--pin+wgrad3_blocks=160 w3b192:--pin+wgrad3_blocks=192' CONFIGS='unet512' REPS=2 bash scripts/ab.sh || exit 1
DIRS='abr3 .' CONFIGS='resnet18_cifar' REPS=3 bash scripts/ab_rev.sh || exit 1
TAG=cifar ARGS="--graph 0" CONFIGS=resnet18_cifar bash scripts/r4_prof.sh || exit 1
O=$R/gpurun_out/r4_prof_cifar_r3; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_resnet18_cifar" -o r -- python3 "$R/abr3/bench.py" --config resnet18_cifar --steps 5 --warmup 2 --graph 0 > "$O/prof.log" 2>&1 || { echo "prof r3 failed"; tail -3 $O/prof.log; exit 1; }
echo "prof r3 cifar $(grep -o '"value": [0-9.]*' $O/prof.log)"
