#!/bin/bash
# Current-state profile of the headline config + host-issue budget:
#   * bench ResNet-50 / ResNet-152 eager with --host_time (host issue time vs GPU time per step),
#     also through a world-size-1 RCCL communicator with the reducer forced on (--rccl1);
#   * --breakdown phase timing;
#   * rocprofv3 kernel trace of ResNet-50 (kernel table + one-step stream analysis).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3_prof; mkdir -p $O
for c in resnet50 resnet152; do
  for r in 0 1; do
    timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 3 --host_time 10 --rccl1 $r --breakdown 3 > $O/host_${c}_rccl$r.log 2>&1 || { echo "fail $c $r"; tail -5 $O/host_${c}_rccl$r.log; exit 1; }
    echo "$c rccl1=$r $(grep -o '"value": [0-9.]*' $O/host_${c}_rccl$r.log) $(grep -o '"host_over_gpu": [0-9.]*' $O/host_${c}_rccl$r.log | head -1)"
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$O/prof_resnet50" -o r -- python3 "$R/bench.py" --steps 5 --warmup 2 > "$R/$O/prof_resnet50.log" 2>&1 || { echo "prof failed"; exit 1; }
echo "prof done $(grep -o '"value": [0-9.]*' $R/$O/prof_resnet50.log)"
