#!/bin/bash
# Register-direct conv epilogue: correctness tests, per-shape conv bench (REPI 0 vs 1), bench A/B.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3_repi; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py tests/test_dual_dgrad_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" $O/tests.log | head -20; exit 1; }
for r in 0 1; do
  timeout -k 10 400 python benchmarks/conv_bench.py --iters 10 --no_miopen --repi $r --only ${ONLY:-fwd} > $O/cb_repi$r.log 2>&1 || { echo "cb fail $r"; tail $O/cb_repi$r.log; exit 1; }
  tail -1 $O/cb_repi$r.log
done
CONFIGS=resnet50 STEPS=20 REPS=2 VARIANTS='base repi0=DLMPI_CONV_REPI=0' bash scripts/env_ab3.sh
