#!/bin/bash
# Persistent tile walk + wgrad row-decode change: GPU tests, per-shape conv bench of the saved
# baseline build (ab_old/) vs the working tree, then DLMPI_CONV_PERSIST A/B on full training steps.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/persist; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread -k "persistent or conv_fwd or conv_dgrad or wgrad" > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" $O/tests.log | head -20; exit 1; }
for i in 1 2; do
  for v in old new; do
    b=benchmarks/conv_bench.py; [ $v = old ] && b=ab_old/benchmarks/conv_bench.py
    for net in resnet50 unet512; do
      timeout -k 10 300 python $b --net $net --no_miopen > $O/cb_${net}_${v}_$i.log 2>&1 || { echo "cb $net $v rc=$?"; tail -5 $O/cb_${net}_${v}_$i.log; exit 1; }
      echo "$net $v #$i $(tail -1 $O/cb_${net}_${v}_$i.log)"
    done
  done
done
for pv in 1 2; do
  DLMPI_CONV_PERSIST=$pv timeout -k 10 300 python benchmarks/conv_bench.py --net resnet50 --no_miopen > $O/cb_resnet50_persist$pv.log 2>&1 || { echo "cb persist rc=$?"; exit 1; }
  echo "resnet50 persist=$pv $(tail -1 $O/cb_resnet50_persist$pv.log)"
done
for i in 1 2; do
  for pv in 0 1 2; do
    DLMPI_CONV_PERSIST=$pv timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_p${pv}_$i.log 2>&1 || { echo "bench rc=$?"; tail -5 $O/bench_p${pv}_$i.log; exit 1; }
    echo "bench persist=$pv #$i $(grep -o '"value": [0-9.]*' $O/bench_p${pv}_$i.log)"
  done
done
