#!/bin/bash
# New GPU tests of this session, then ResNet-18 CIFAR (the reference's own config): round-1-end tree
# (abr1/, built in-tree) vs the working tree, eager and hipGraph, alternating order, plus one
# kernel trace of each build (eager) for per-step kernel counts.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3_cifar_ab; mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -x -v -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1
  rc=$?; tail -3 $O/tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" $O/tests.log | head -20; exit 1; }
fi
for i in 1 2 3; do
  order="old new"; [ $((i % 2)) -eq 0 ] && order="new old"
  for v in $order; do
    d=$R; [ $v = old ] && d=$R/abr1
    for g in 0 1; do
      (cd $d && timeout -k 10 300 python bench.py --config resnet18_cifar --graph $g --steps 100 --warmup 5) > $O/${v}_g${g}_$i.log 2>&1 || { echo "fail $v g$g"; tail -5 $O/${v}_g${g}_$i.log; exit 1; }
      echo "$v graph=$g #$i $(grep -o '"value": [0-9.]*' $O/${v}_g${g}_$i.log)"
    done
  done
done
cd /tmp && export TMPDIR=/tmp
for v in old new; do
  d=$R; [ $v = old ] && d=$R/abr1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$O/prof_$v" -o r -- python3 "$d/bench.py" --config resnet18_cifar --steps 20 --warmup 2 > "$R/$O/prof_$v.log" 2>&1 || { echo "prof $v failed"; exit 1; }
done
echo done
