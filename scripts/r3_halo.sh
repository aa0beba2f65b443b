#!/bin/bash
# 2-D halo tiles for 3x3 stride-1 convs: kernel tests, per-shape timing on/off, bench A/B.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3_halo; mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --timeout 180 --timeout-method thread tests/test_kernels_gpu.py tests/test_models_gpu.py tests/test_fuse_apply_gpu.py > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -ne 0 ] && { grep -E "^FAILED|^E  " $O/tests.log | head -20; exit 1; }
for shp in 256,56,56,64,64,3,1,1 256,28,28,128,128,3,1,1 256,14,14,256,256,3,1,1 256,7,7,512,512,3,1,1 16,512,512,64,64,3,1,1 16,256,256,128,128,3,1,1 16,128,128,256,256,3,1,1 16,64,64,512,512,3,1,1 16,32,32,1024,1024,3,1,1; do
  for ps in fwd dgrad; do
    for m in 1 0; do
      DLMPI_CONV_HALO=$m timeout -k 5 120 python benchmarks/conv_one.py --shape $shp --pass $ps --iters 10 2>&1 | grep -E "^(fwd|dgrad)" | sed "s/^/halo=$m /" >> $O/times.log || { echo "fail $shp $m"; exit 1; }
    done
  done
done
cat $O/times.log
CONFIGS="resnet50 unet512" STEPS=10 REPS=2 VARIANTS='base h0=DLMPI_CONV_HALO=0' bash scripts/env_ab3.sh
