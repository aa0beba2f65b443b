#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3_c512; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -k "stream1x1" -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" $O/tests.log | head -20; exit 1; }
for v in 0 1; do
  DLMPI_CONV_STREAM_C512=$v timeout -k 10 400 python benchmarks/conv_bench.py --iters 10 --no_miopen --only fwd > $O/cb_c512_$v.log 2>&1 || { echo "cb fail $v"; tail $O/cb_c512_$v.log; exit 1; }
  grep '"shape": \[256, 7, 7, 512, 2048' $O/cb_c512_$v.log; tail -1 $O/cb_c512_$v.log
done
CONFIGS=resnet50 STEPS=20 REPS=2 VARIANTS='base c0=DLMPI_CONV_STREAM_C512=0' bash scripts/env_ab3.sh
