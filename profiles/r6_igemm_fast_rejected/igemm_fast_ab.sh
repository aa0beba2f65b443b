# conv_igemm_kernel scalar-base staging: bit-identity tests, per-shape timing (production dispatch), bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT && export HSA_ENABLE_IPC_MODE_LEGACY=0 && O=gpurun_out/igf && mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "igemm_fast or pipelined or conv_fwd or conv_dgrad or halo" > $O/tests.log 2>&1 && tail -2 $O/tests.log || exit 1
for sh in 256,56,56,64,256,1,1,0 256,56,56,256,64,1,1,0 256,28,28,512,128,1,1,0 256,28,28,128,512,1,1,0 256,14,14,1024,256,1,1,0 256,56,56,256,512,1,2,0 256,28,28,128,128,3,1,1; do
  for ps in fwd dgrad; do
    for v in 0 1; do
      r=$(timeout -k 10 60 python benchmarks/conv_one.py --shape $sh --pass $ps --iters 30 --set set_igemm_fast=$v 2>/dev/null | tail -1) || exit 1
      echo "fast=$v $r"
    done
  done
done > $O/shapes.log && cat $O/shapes.log &&
OUT=$O/ab VARIANTS="base slow:--pin+igemm_fast=0" CONFIGS="resnet50 unet512" REPS=3 bash scripts/ab.sh
