#!/bin/bash
# fp32 precision path on the GPU: its kernel tests (vs fp64) + the kernel suite, then a rocprofv3
# kernel trace of ResNet-18 CIFAR training with --precision fp32 (every kernel must be ours), and
# the throughput of that path next to bf16.  Output: gpurun_out/${1:-r2_fp32}/
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r2_fp32}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd "$R"
[ -n "$SKIP_TESTS" ] || timeout -k 10 600 python -u -m pytest tests/test_fp32_gpu.py tests/test_kernels_gpu.py -x -v -m gpu --timeout 180 \
  --timeout-method thread > $O/tests.log 2>&1
rc=$?
grep -E "passed|failed|error" $O/tests.log | tail -3
[ $rc -eq 0 ] || { grep -E "FAILED|Error|error|assert" $O/tests.log | head -30; exit 1; }
for prec in fp32 bf16; do
  timeout -k 10 240 python pytorch/resnet/main.py --arch resnet18 --precision $prec \
    --synthetic --batch_size 128 --benchmark_steps 50 > $O/cifar_$prec.log 2>&1 || { tail -20 $O/cifar_$prec.log; exit 1; }
  tail -2 $O/cifar_$prec.log
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o r -- python3 $R/pytorch/resnet/main.py \
  --arch resnet18 --precision fp32 --synthetic --batch_size 128 --benchmark_steps 200 --graph 0 > $O/prof.log 2>&1 \
  || { tail -20 $O/prof.log; exit 1; }
cd "$R" && python scripts/prof_summary.py $(ls $O/prof/*.db $O/prof/*/*.db 2>/dev/null | head -1) --step-kernel sgd_kernel --window 0.2 --top 40 > $O/prof_summary.txt 2>&1; head -40 $O/prof_summary.txt
