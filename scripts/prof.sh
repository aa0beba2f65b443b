#!/bin/bash
# Kernel-trace profiles of the training step (rocprofv3 --kernel-trace --stats; no counters): one
# per CONFIG (extra bench arguments: ARGS, e.g. --graph 0).  Digest on the CPU side with scripts/prof_summary.py and scripts/step_analysis.py.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/prof${TAG:+_$TAG}; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp
for c in ${CONFIGS:-unet512 resnet50}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_$c" -o r -- python3 "$R/bench.py" --config $c --steps ${STEPS:-5} --warmup 2 ${ARGS} > "$O/prof_$c.log" 2>&1 || { echo "prof $c failed"; tail -3 "$O/prof_$c.log"; exit 1; }
  echo "prof $c $(grep -o '"value": [0-9.]*' $O/prof_$c.log)"
done
exit 0
