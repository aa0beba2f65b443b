#!/bin/bash
# GPU pass.  STEPS selects what runs (default: kernels models smoke bench prof convbench).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
STEPS=${STEPS:-"kernels models smoke bench prof convbench"}
run() { local name=$1; shift; local t=$1; shift; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; if [ $rc -gt 1 ]; then exit $rc; fi; }
for s in $STEPS; do
  case $s in
    kernels) run kernels 900 python -m pytest tests/test_kernels_gpu.py -q -m gpu ;;
    models) run models 600 python -m pytest tests/test_models_gpu.py -q -m gpu ;;
    graphs) run graphs 600 python -m pytest tests/test_graphs_gpu.py -q -m gpu ;;
    allgpu) run allgpu 1500 python -m pytest tests -q -m gpu ;;
    benchgraph) run benchgraph 400 python bench.py --steps 10 --warmup 3 --graph 1 ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 400 python bench.py --steps 10 --warmup 3 ;;
    baseline) run baseline 400 python benchmarks/torch_baseline.py --steps 10 --warmup 3 ;;
    convbench) run convbench 600 python benchmarks/conv_bench.py ;;
    configs)
      for c in ${CONFIGS:-resnet18_cifar resnet152 unet512 unet1024}; do
        run "cfg_${c}_ours" 600 python bench.py --config $c --steps 10 --warmup 3
        run "cfg_${c}_graph" 600 python bench.py --config $c --steps 10 --warmup 3 --graph 1
        if [ -z "$SKIP_TORCH" ]; then run "cfg_${c}_torch" 600 python benchmarks/torch_baseline.py --config $c --steps 10 --warmup 3; fi
      done ;;
    prof)
      ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o bench --output-format csv -- python "$R/bench.py" --steps 5 --warmup 2 > "$R/gpurun_out/prof.log" 2>&1 ); echo "prof rc=$?" ;;
  esac
done
