#!/bin/bash
# stream-K: kernel tests, per-shape A/B (DLMPI_CONV_SK=0 vs auto), bench A/B
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu --timeout 180 --timeout-method thread -k "stream_k or conv_fwd or conv_dgrad or split" > gpurun_out/sk_tests.log 2>&1
rc=$?; echo "tests rc=$rc: $(tail -1 gpurun_out/sk_tests.log)"; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" gpurun_out/sk_tests.log | head -20; exit 1; }
for v in 0 1; do
  for spec in "256,14,14,1024,256,1,1,0 fwd" "256,14,14,256,1024,1,1,0 dgrad" "256,28,28,512,128,1,1,0 fwd" "256,28,28,128,128,3,1,1 fwd" "256,28,28,128,128,3,1,1 dgrad" "256,7,7,512,2048,1,1,0 fwd" "256,7,7,2048,512,1,1,0 dgrad" "256,14,14,256,256,3,1,1 fwd" "256,7,7,512,512,3,1,1 fwd"; do
    set -- $spec
    r=$(DLMPI_CONV_SK=$v timeout -k 10 60 python benchmarks/conv_one.py --shape $1 --pass $2 --iters 30 2>/dev/null | tail -1) || { echo fail; exit 1; }
    echo "sk=$v | $r"
  done
done
AB_SETS="DLMPI_CONV_SK=0;DLMPI_CONV_SK=1" AB_REPS=2 bash scripts/multi_ab.sh
