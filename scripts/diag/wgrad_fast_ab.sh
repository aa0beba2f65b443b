set -o pipefail
cd $GRAFT_REPO_ROOT && export HSA_ENABLE_IPC_MODE_LEGACY=0 && mkdir -p gpurun_out/wf
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "wgrad" > gpurun_out/wf/tests.log 2>&1 && tail -3 gpurun_out/wf/tests.log &&
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_wgrad_defer_gpu.py > gpurun_out/wf/tests2.log 2>&1 && tail -2 gpurun_out/wf/tests2.log &&
timeout -k 10 400 python -u benchmarks/wgrad_lab.py --net resnet50 --rounds 3 --arms "slow:set_wgrad_fast=0;fast:set_wgrad_fast=1" > gpurun_out/wf/lab.log 2>&1 && tail -3 gpurun_out/wf/lab.log &&
OUT=gpurun_out/wf/ab VARIANTS="base slow:--pin+wgrad_fast=0" CONFIGS="resnet50 unet512" REPS=3 bash scripts/ab.sh
