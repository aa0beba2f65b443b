#!/bin/bash
# Kernel-trace profile of the same config from two built trees (DIRS), for per-kernel A/B.
R=${GRAFT_REPO_ROOT:-$(pwd)}
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp
for d in ${DIRS:-abh .}; do
  tag=$(echo $d | tr -d './'); tag=${tag:-head}
  O=$R/gpurun_out/profab_$tag; mkdir -p $O
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof" -o r -- python3 "$R/$d/bench.py" --config ${CONFIG:-resnet50} --steps 3 --warmup 2 > "$O/prof.log" 2>&1 || { echo "prof $d failed"; tail -3 $O/prof.log; exit 1; }
  echo "prof $tag $(grep -o '"value": [0-9.]*' $O/prof.log)"
done
