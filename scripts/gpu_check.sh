#!/bin/bash
# Round-4 GPU check of the working tree: conv lab (pass 2), the GPU test suite, smoke, and the headline
# benches.  Every GPU step has its own time limit; the script stops at the first failure.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && export HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out/gpu_check${TAG:+_$TAG}; mkdir -p $O
if [ -z "$NOLAB" ]; then
  timeout -k 10 300 ./benchmarks/conv_lab 3 ${SHAPES} > $O/lab.log 2>&1 || { echo lab failed; tail -5 $O/lab.log; exit 1; }
  echo "lab OK=$(grep -c ' OK ' $O/lab.log) BAD=$(grep -c ' BAD ' $O/lab.log)"
fi
if [ -z "$NOTEST" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 180 --timeout-method thread ${TESTS} > $O/tests.log 2>&1
  rc=$?; tail -1 $O/tests.log
  if [ $rc -ne 0 ]; then grep -E "^FAILED|^ERROR|Error" $O/tests.log | head -20; exit 1; fi
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail -5 $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log
fi
for c in ${CONFIGS:-resnet50 unet512}; do
  timeout -k 10 300 python bench.py --config $c > $O/bench_$c.log 2>&1 || { echo "bench $c failed"; tail -5 $O/bench_$c.log; exit 1; }
  echo "bench $c $(grep -o '"value": [0-9.]*' $O/bench_$c.log) $(grep -o '"ms_per_step": [0-9.]*' $O/bench_$c.log)"
done
exit 0
