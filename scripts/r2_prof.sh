#!/bin/bash
# rocprofv3 kernel trace of bench.py (ResNet-50 default, or PROF_CONFIG) -> gpurun_out/${PROF_OUT:-r2_prof}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out/${PROF_OUT:-r2_prof}; mkdir -p $O
for c in ${PROF_CONFIGS:-resnet50}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/$c" -o r -- python3 "$R/bench.py" --config $c --steps 5 --warmup 2 > "$O/$c.log" 2>&1 || { echo "prof $c failed"; tail -5 "$O/$c.log"; exit 1; }
  echo "$c $(grep -o '"value": [0-9.]*' $O/$c.log)"
done
