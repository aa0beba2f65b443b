#!/bin/bash
# rocprofv3 kernel stats of bench.py under two environment settings: PROF_A / PROF_B (VAR=val pairs)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out/${PROF_OUT:-prof2}
mkdir -p $O
for tag in a b; do
  if [ $tag = a ]; then E="$PROF_A"; else E="$PROF_B"; fi
  env $E timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/$tag" -o r -- python3 "$R/bench.py" --config ${PROF_CONFIG:-resnet50} --steps 5 --warmup 2 > "$O/$tag.log" 2>&1 || { echo "prof $tag failed"; tail -5 "$O/$tag.log"; exit 1; }
  echo "$tag ($E): $(grep -o '"value": [0-9.]*' $O/$tag.log)"
done
