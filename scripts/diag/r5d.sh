R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/convtab_r5
timeout -k 10 400 python -u benchmarks/conv_bench.py --net resnet50 --iters 20 > gpurun_out/convtab_r5/resnet50.log 2>&1 || { echo convtab failed; tail -5 gpurun_out/convtab_r5/resnet50.log; exit 1; }
echo convtab ok
CONFIGS="resnet50 unet512 resnet18_cifar" TAG=r5d bash scripts/copytrace.sh > gpurun_out/ct.log 2>&1 || { echo copytrace failed; tail gpurun_out/ct.log; exit 1; }
echo copytrace ok
CONFIGS="resnet50 unet512 resnet18_cifar" TAG=r5d STEPS=10 bash scripts/prof.sh
