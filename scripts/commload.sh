#!/bin/bash
# Comm-load rehearsal sweep: world-1 RCCL reducer (--rccl1) vs the modeled 8-rank
# all-reduce load with 8 / 16 / 32 channels, ResNet-50 and ResNet-152, same box.  Output:
# gpurun_out/commload/
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && export HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out/commload; mkdir -p $O
for c in ${CONFIGS:-resnet50 resnet152}; do
  for v in rccl1 8 16 32; do
    if [ $v = rccl1 ]; then args="--rccl1 1 --breakdown 3"; else args="--rehearse $v"; fi
    timeout -k 10 300 python bench.py --config $c --steps ${STEPS:-15} --warmup 5 $args > $O/${c}_$v.log 2>&1 || { echo "fail $c $v"; tail -5 $O/${c}_$v.log; exit 1; }
    echo "$c $v $(grep -o '"value": [0-9.]*' $O/${c}_$v.log) $(grep -o '"ms_per_step": [0-9.]*' $O/${c}_$v.log) $(grep -o '"comm_exposed_ms": [0-9.a-z]*' $O/${c}_$v.log) $(grep -o '"modeled_allreduce_us_per_step": [0-9.]*' $O/${c}_$v.log) $(grep -o '"dgrad_stream_blocks": [0-9]*' $O/${c}_$v.log)"
  done
done
