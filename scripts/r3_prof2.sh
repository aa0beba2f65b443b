#!/bin/bash
# rocprofv3 kernel trace of the default ResNet-50 bench step (kernel table + one-step analysis input).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/${1:-r3_prof2}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$O/prof_resnet50" -o r -- python3 "$R/bench.py" --steps 5 --warmup 2 > "$R/$O/prof_resnet50.log" 2>&1 || { echo "prof failed"; tail -5 "$R/$O/prof_resnet50.log"; exit 1; }
echo "prof done $(grep -o '"value": [0-9.]*' $R/$O/prof_resnet50.log)"
