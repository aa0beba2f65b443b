#!/bin/bash
# GPU tests of the operand prologues, then bench.py A/B: deferred BN passes on (default) vs off.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/dab
export HSA_ENABLE_IPC_MODE_LEGACY=0
TESTS=${TESTS:-"tests/test_kernels_gpu.py tests/test_models_gpu.py tests/test_graphs_gpu.py tests/test_ddp_rccl_gpu.py"}
if [ "$TESTS" != none ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -x -q -m gpu --timeout 180 --timeout-method thread > gpurun_out/dab/tests.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/dab/tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/dab/tests.log | head; exit 1; }
fi
for i in $(seq 1 ${AB_REPS:-2}); do
  for c in ${AB_CONFIGS:-resnet50 unet512}; do
    for v in 1 0; do
      DLMPI_DEFER_BN_FWD=$v DLMPI_DEFER_BN_BWD=$v timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 > gpurun_out/dab/${c}_d${v}_$i.log 2>&1 || { echo "bench $c $v failed"; tail -20 gpurun_out/dab/${c}_d${v}_$i.log; exit 1; }
      echo "$c defer=$v #$i $(grep -o '"value": [0-9.]*' gpurun_out/dab/${c}_d${v}_$i.log)"
    done
  done
done
