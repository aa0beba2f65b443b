# deferred-dz (PA 2) weight-gradient fast staging: bit-identity tests, then a same-box A/B
set -o pipefail
cd $GRAFT_REPO_ROOT && export HSA_ENABLE_IPC_MODE_LEGACY=0 && O=gpurun_out/wpa2 && mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_wgrad_fast_gpu.py tests/test_kernels_gpu.py -k "wgrad" > $O/tests.log 2>&1 && tail -2 $O/tests.log || exit 1
OUT=$O/ab VARIANTS="base pa0:--pin+wgrad_fast=1" CONFIGS="unet512 resnet50" REPS=3 bash scripts/ab.sh
