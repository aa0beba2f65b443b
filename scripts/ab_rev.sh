#!/bin/bash
# Same-box A/B of git revisions: every DIR (a built worktree under the repo root, "." = this tree)
# runs bench.py for every CONFIG, REPS times, alternating the order per repetition.
#   DIRS="abr3 ." CONFIGS="resnet50 unet512" REPS=3 STEPS=20 OUT=gpurun_out/ab_rev
R=${GRAFT_REPO_ROOT:-$(pwd)}
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/${OUT:-gpurun_out/ab_rev}; mkdir -p $O
for i in $(seq 1 ${REPS:-3}); do
  ds="$DIRS"; [ $((i % 2)) -eq 0 ] && ds=$(echo $DIRS | tr ' ' '\n' | tac | tr '\n' ' ')
  for d in $ds; do
    for c in ${CONFIGS:-resnet50}; do
      tag=$(echo $d | tr -d './'); tag=${tag:-head}
      log=$O/${c}_${tag}_$i.log
      (cd $R/$d && timeout -k 10 ${TLIM:-300} python bench.py --config $c --steps ${STEPS:-20} --warmup ${WARMUP:-5} ${ARGS} > $log 2>&1) || { echo "fail $d $c"; tail -5 $log; exit 1; }
      echo "$c $tag #$i $(grep -o '"value": [0-9.]*' $log)"
    done
  done
done
