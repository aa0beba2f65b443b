#!/bin/bash
# Full-training-step A/B of two builds on the same box: ab_old/ (a saved, separately built copy of
# the package + bench.py, e.g. `git archive HEAD deeplearning_mpi_amd bench.py | tar -x -C ab_old`)
# vs the working tree, alternating.  TESTS="..." runs GPU tests of the working tree first.
# AB_CONFIGS="resnet50 unet512" AB_REPS=3
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/bab
export HSA_ENABLE_IPC_MODE_LEGACY=0
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/bab/tests.log 2>&1
  rc=$?; echo "tests rc=$rc"; [ $rc -ne 0 ] && { tail -40 gpurun_out/bab/tests.log; exit 1; }
fi
for i in $(seq 1 ${AB_REPS:-3}); do
  for c in ${AB_CONFIGS:-resnet50}; do
    # alternate which build runs first: a fixed order biases the A/B by ~0.4 % (profiles/r1_cast_transpose)
    order="old new"; [ $((i % 2)) -eq 0 ] && order="new old"
    for v in $order; do
      b=bench.py; [ $v = old ] && b=ab_old/bench.py
      timeout -k 10 300 python $b --config $c --steps ${AB_STEPS:-10} --warmup 3 > gpurun_out/bab/${c}_${v}_$i.log 2>&1 || { echo "bench $c $v rc=$?"; tail -20 gpurun_out/bab/${c}_${v}_$i.log; exit 1; }
      echo "$c $v #$i $(grep -o '"value": [0-9.]*' gpurun_out/bab/${c}_${v}_$i.log)"
    done
  done
done
