#!/bin/bash
# 64x256 weight-gradient tile for Ko <= 64: correctness with the tile forced on, per-shape conv bench
# for DLMPI_WGRAD_WIDE=0/1/2, then full training steps 0 vs 1 vs 2.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/wgwide; mkdir -p $O
DLMPI_WGRAD_WIDE=${TW:-2} timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_benchscale_gpu.py -x -q -m gpu --timeout 180 --timeout-method thread -k "wgrad or benchscale or bench_scale" > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" $O/tests.log | head -20; exit 1; }
for v in ${WVALS:-0 1 2}; do
  for net in resnet50 unet512; do
    DLMPI_WGRAD_WIDE=$v timeout -k 10 300 python benchmarks/conv_bench.py --net $net --no_miopen > $O/cb_${net}_w$v.log 2>&1 || { echo "cb $net $v rc=$?"; tail -5 $O/cb_${net}_w$v.log; exit 1; }
    echo "$net wide=$v $(tail -1 $O/cb_${net}_w$v.log)"
  done
done
for i in 1 2; do
  for c in resnet50 unet512; do
    for v in ${WVALS:-0 1 2}; do
      DLMPI_WGRAD_WIDE=$v timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 > $O/bench_${c}_w${v}_$i.log 2>&1 || { echo "bench rc=$?"; tail -5 $O/bench_${c}_w${v}_$i.log; exit 1; }
      echo "bench $c wide=$v #$i $(grep -o '"value": [0-9.]*' $O/bench_${c}_w${v}_$i.log)"
    done
  done
done
