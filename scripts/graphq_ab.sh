#!/bin/bash
# hipGraph replay vs eager for ResNet-50 under the HIP runtime's graph-execution knobs
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/graphq && export HSA_ENABLE_IPC_MODE_LEGACY=0
for i in 1 2; do
  for v in "eager" "graph" "graph DEBUG_CLR_GRAPH_PACKET_CAPTURE=0" "graph DEBUG_HIP_FORCE_GRAPH_QUEUES=4" "graph DEBUG_HIP_FORCE_GRAPH_QUEUES=2"; do
    set -- $v; mode=$1; shift
    g=0; [ $mode = graph ] && g=1
    tag=$(echo "$v" | tr ' =' '_-')
    env "$@" timeout -k 10 300 python bench.py --config ${CFG:-resnet50} --graph $g --steps 20 --warmup 5 > gpurun_out/graphq/${tag}_$i.log 2>&1 || { echo "bench $v rc=$?"; tail -5 gpurun_out/graphq/${tag}_$i.log; exit 1; }
    echo "$v #$i $(grep -o '"value": [0-9.]*' gpurun_out/graphq/${tag}_$i.log)"
  done
done
