#!/bin/bash
# Streaming dgrad v3 (48-row 6-wave tiles for K = 256) + stem wgrad on the main stream: tests, timings,
# ResNet-50 / ResNet-152 A/B (alternating): base | k32 (K=256 on 32-row tiles) | t0 (stem wgrad on side)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3_dgs3; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_dgrad_stream_gpu.py tests/test_ddp_rccl_gpu.py tests/test_comm_ordering_gpu.py tests/test_graphs_gpu.py -x -q --timeout 180 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -ne 0 ] && { grep -E "^FAILED|^ERROR|Error" $O/tests.log | head -20; exit 1; }
timeout -k 10 300 python benchmarks/dgrad_stream_bench.py > $O/times.log 2>&1 || { tail $O/times.log; exit 1; }
cat $O/times.log
DLMPI_DGS_K256_ROWS=32 timeout -k 10 300 python benchmarks/dgrad_stream_bench.py > $O/times_k32.log 2>&1 || { tail $O/times_k32.log; exit 1; }
grep -E "layer2|layer3" $O/times_k32.log
for i in 1 2; do
  for v in base k32 t0; do
    unset DLMPI_DGS_K256_ROWS DLMPI_WGRAD_TAIL_MAIN
    case $v in k32) export DLMPI_DGS_K256_ROWS=32;; t0) export DLMPI_WGRAD_TAIL_MAIN=0;; esac
    for c in resnet50 resnet152; do
      timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 > $O/${c}_${v}_$i.log 2>&1 || { echo "bench $c $v failed"; tail -5 $O/${c}_${v}_$i.log; exit 1; }
      echo "$c $v #$i $(grep -o '"value": [0-9.]*' $O/${c}_${v}_$i.log)"
    done
  done
done
