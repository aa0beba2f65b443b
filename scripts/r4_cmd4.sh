#!/bin/bash
# Round-4: flush-granularity A/B (ResNet-50), UNet round 3 vs HEAD (same box), comm-load rehearsal.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
VARIANTS='base b4:--pin+wgrad_batch=4 b8:--pin+wgrad_batch=8 small:--pin+defer_direct=0 nodefer:--pin+defer=0' CONFIGS=resnet50 REPS=2 bash scripts/ab.sh || exit 1
DIRS='abr3 .' CONFIGS='unet512 unet1024' REPS=2 bash scripts/ab_rev.sh || exit 1
bash scripts/r4_commload.sh || exit 1
