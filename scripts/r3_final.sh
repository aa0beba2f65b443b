#!/bin/bash
# End-of-session validation (round 3) on one box: full GPU suite, smoke, every BASELINE.json config through
# bench.py, and the 2-rank DDP rehearsal (gloo transport, both ranks on device 0).
# Output: gpurun_out/r3_final/
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3_final; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 180 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -2 $O/gpu_tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" $O/gpu_tests.log | head -20; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for c in resnet50 resnet152 unet512 unet1024 resnet18_cifar; do
  st=20; [ $c = unet1024 ] && st=10
  timeout -k 10 400 python bench.py --config $c --steps $st --warmup 5 > $O/bench_$c.log 2>&1 || { echo "bench $c rc=$?"; tail -5 $O/bench_$c.log; exit 1; }
  echo "$c $(grep -o '"value": [0-9.]*' $O/bench_$c.log)"
done
timeout -k 10 400 python bench.py --config resnet18_cifar --graph 1 --steps 50 --warmup 5 > $O/bench_resnet18_cifar_graph.log 2>&1 || { echo "graph bench rc=$?"; exit 1; }
echo "resnet18_cifar graph $(grep -o '"value": [0-9.]*' $O/bench_resnet18_cifar_graph.log)"
export DLMPI_GLOO_DEVICE=cuda
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29532 \
  bench.py --gpus 2 --steps 4 --warmup 2 --batch 64 --backend gloo > $O/bench2.log 2>&1 || { echo "bench2 rc=$?"; tail -5 $O/bench2.log; exit 1; }
echo "2-rank rehearsal $(grep -o '"n_gpus": [0-9]*' $O/bench2.log)"
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 \
  tests/ddp_gpu_rehearsal.py > $O/ddp2.log 2>&1 || { echo "ddp2 rc=$?"; tail -5 $O/ddp2.log; exit 1; }
echo "ddp rehearsal ok"
# rocprof kernel trace of the headline config (kernel table + one-step analysis)
cd /tmp && export TMPDIR=/tmp && unset DLMPI_GLOO_DEVICE
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$O/prof_resnet50" -o r -- python3 "$R/bench.py" --steps 5 --warmup 2 > "$R/$O/prof_resnet50.log" 2>&1 || { echo "prof failed"; exit 1; }
echo "prof done $(grep -o '"value": [0-9.]*' $R/$O/prof_resnet50.log)"
