#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -m pytest tests -q -m gpu -x > gpurun_out/allgpu.log 2>&1; echo "allgpu rc=$?"
for nt in 0 1; do
  DLMPI_NT_STORE=$nt timeout -k 10 400 python bench.py --steps 20 --warmup 3 > gpurun_out/bench_nt$nt.log 2>&1 || exit 1
  DLMPI_NT_STORE=$nt timeout -k 10 400 python benchmarks/conv_bench.py --iters 10 --no_miopen --only fwd > gpurun_out/cb_fwd_nt$nt.log 2>&1 || exit 1
done
DLMPI_NT_STORE=0 timeout -k 10 400 python bench.py --steps 20 --warmup 3 > gpurun_out/bench_nt0b.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o bench --output-format csv -- python "$R/bench.py" --steps 5 --warmup 2 > "$R/gpurun_out/prof.log" 2>&1; echo "prof rc=$?"
