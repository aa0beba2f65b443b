#!/bin/bash
# Same-box A/B driver for bench.py (the one parameterised replacement of the per-experiment r1_*/r2_*/
# r3_* scripts; their results stay in profiles/).  Runs every VARIANT on every CONFIG, REPS times,
# alternating the variant order per repetition (cdna_hip_programming.md §5.4 rule 24), and prints one
# line per run with the bench value.
#   VARIANTS="NAME[=ENV=VAL[,ENV2=VAL2]][:bench args with '+' for spaces] ..."   (base = no change)
#   CONFIGS="resnet50 unet512" REPS=3 STEPS=20 OUT=gpurun_out/ab
# e.g. VARIANTS="base ch8:--rehearse+8 ch16:--rehearse+16" CONFIGS=resnet50 bash scripts/ab.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && export HSA_ENABLE_IPC_MODE_LEGACY=0
O=${OUT:-gpurun_out/ab}; mkdir -p $O
for i in $(seq 1 ${REPS:-3}); do
  vs="$VARIANTS"; [ $((i % 2)) -eq 0 ] && vs=$(echo $VARIANTS | tr ' ' '\n' | tac | tr '\n' ' ')
  for v in $vs; do
    spec=${v%%:*}; args=""; [ "$spec" != "$v" ] && args=$(echo ${v#*:} | tr '+' ' ')
    name=${spec%%=*}; envs=${spec#*=}; [ "$name" = "$spec" ] && envs=""
    for c in ${CONFIGS:-resnet50}; do
      log=$O/${c}_${name}_$i.log
      env $(echo $envs | tr ',' ' ') timeout -k 10 ${TLIM:-300} python bench.py --config $c --steps ${STEPS:-20} \
        --warmup ${WARMUP:-5} $args > $log 2>&1 || { echo "fail $name $c"; tail -5 $log; exit 1; }
      echo "$c $name #$i $(grep -o '"value": [0-9.]*' $log) $(grep -o '"comm_exposed_ms": [0-9.a-z]*' $log)"
    done
  done
done
