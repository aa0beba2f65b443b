#!/bin/bash
# GPU tests, then an A/B of one environment knob on full bench.py training steps, alternating
# values on the same box: AB_VAR=NAME AB_VALS="0 1" AB_CONFIGS="resnet50 unet512" AB_REPS=2
# TESTS="tests/..." (default: kernel + model + graph tests; TESTS=none skips them).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/ab
export HSA_ENABLE_IPC_MODE_LEGACY=0
TESTS=${TESTS:-"tests/test_kernels_gpu.py tests/test_models_gpu.py tests/test_graphs_gpu.py"}
if [ "$TESTS" != none ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/ab/tests.log 2>&1
  rc=$?; echo "tests rc=$rc"; [ $rc -ne 0 ] && { tail -40 gpurun_out/ab/tests.log; exit 1; }
fi
for i in $(seq 1 ${AB_REPS:-2}); do
  for c in ${AB_CONFIGS:-resnet50}; do
    for v in ${AB_VALS:-0 1}; do
      env "$AB_VAR=$v" timeout -k 10 300 python bench.py --config $c --steps ${AB_STEPS:-10} --warmup 3 > gpurun_out/ab/${c}_${AB_VAR}_${v}_$i.log 2>&1 || { echo "bench $c $v rc=$?"; tail -20 gpurun_out/ab/${c}_${AB_VAR}_${v}_$i.log; exit 1; }
      echo "$c $AB_VAR=$v #$i $(grep -o '"value": [0-9.]*' gpurun_out/ab/${c}_${AB_VAR}_${v}_$i.log)"
    done
  done
done
