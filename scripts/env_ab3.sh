#!/bin/bash
# Environment-knob A/B on one box, alternating order: CONFIG (bench preset), GRAPH (0/1),
# VARIANTS="NAME=ENV=VAL[,ENV2=VAL2] ..." (NAME=base for none), REPS.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/env_ab3; mkdir -p $O
for i in $(seq 1 ${REPS:-3}); do
  vs="$VARIANTS"; [ $((i % 2)) -eq 0 ] && vs=$(echo $VARIANTS | tr ' ' '\n' | tac | tr '\n' ' ')
  for v in $vs; do
    name=${v%%=*}; envs=${v#*=}; [ "$name" = "$v" ] && envs=""
    for c in ${CONFIGS:-resnet18_cifar}; do
      env $(echo $envs | tr ',' ' ') timeout -k 10 300 python bench.py --config $c --graph ${GRAPH:-0} --steps ${STEPS:-50} --warmup 5 > $O/${c}_${name}_$i.log 2>&1 || { echo "fail $name $c"; tail -5 $O/${c}_${name}_$i.log; exit 1; }
      echo "$c $name #$i $(grep -o '"value": [0-9.]*' $O/${c}_${name}_$i.log)"
    done
  done
done
