#!/bin/bash
# bench.py eager vs --graph 1 on the same box, alternating: AB_CONFIGS="resnet50 unet512" AB_REPS=2
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/gab
export HSA_ENABLE_IPC_MODE_LEGACY=0
for i in $(seq 1 ${AB_REPS:-2}); do
  for c in ${AB_CONFIGS:-resnet50}; do
    for g in 0 1; do
      timeout -k 10 300 python bench.py --config $c --steps ${AB_STEPS:-20} --warmup 5 --graph $g > gpurun_out/gab/${c}_g${g}_$i.log 2>&1 || { echo "bench $c g=$g failed"; tail -20 gpurun_out/gab/${c}_g${g}_$i.log; exit 1; }
      echo "$c graph=$g #$i $(grep -o '"value": [0-9.]*' gpurun_out/gab/${c}_g${g}_$i.log)"
    done
  done
done
