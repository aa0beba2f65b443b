#!/bin/bash
# bench.py A/B over several environment settings (space-separated VAR=val lists, ';'-separated),
# alternating on one box: AB_SETS="A=0 B=0;A=1 B=0" AB_REPS=2 AB_CONFIG=resnet50 AB_STEPS=20
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/mab
export HSA_ENABLE_IPC_MODE_LEGACY=0
IFS=';' read -ra SETS <<< "$AB_SETS"
for i in $(seq 1 ${AB_REPS:-2}); do
  for s in "${SETS[@]}"; do
    tag=$(echo "$s" | tr ' =' '_-')
    env $s timeout -k 10 300 python bench.py --config ${AB_CONFIG:-resnet50} --steps ${AB_STEPS:-20} --warmup 3 > gpurun_out/mab/${tag}_$i.log 2>&1 || { echo "bench [$s] rc=$?"; tail -20 gpurun_out/mab/${tag}_$i.log; exit 1; }
    echo "[$s] #$i $(grep -o '"value": [0-9.]*' gpurun_out/mab/${tag}_$i.log)"
  done
done
