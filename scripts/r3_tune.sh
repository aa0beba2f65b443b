#!/bin/bash
# Conv autotuner: full GPU suite (no -x: every failure in one run), ResNet-50 / ResNet-152 A/B
# (autotune on/off), then the current-state profile.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3_tune; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 180 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log
if [ $rc -ne 0 ]; then grep -E "^FAILED|^ERROR" $O/tests.log | head -30; [ $rc -ge 124 ] && exit 1; fi
DLMPI_CONV_AUTOTUNE_LOG=1 timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $O/tune_log.txt 2>&1 || { echo tune log fail; tail -5 $O/tune_log.txt; exit 1; }
CONFIGS="resnet50 resnet152" STEPS=20 REPS=2 VARIANTS='base at0=DLMPI_CONV_AUTOTUNE=0' bash scripts/env_ab3.sh || exit 1
bash scripts/r3_prof.sh
