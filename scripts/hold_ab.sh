#!/bin/bash
# A/B: cross-stream buffer lifetimes held until the backward join (DLMPI_STREAM_HOLD=1) vs record_stream.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/hold
export HSA_ENABLE_IPC_MODE_LEGACY=0
for i in 1 2; do
  for h in 1 0; do
    DLMPI_STREAM_HOLD=$h timeout -k 10 300 python bench.py --config unet1024 --steps 10 --warmup 3 --mem 1 \
      > gpurun_out/hold/unet1024_h${h}_$i.log 2>&1 || exit 1
    echo "unet1024 hold=$h #$i $(grep -o '"value": [0-9.]*' gpurun_out/hold/unet1024_h${h}_$i.log) $(grep -o 'peak_reserved_gb": [0-9.]*' gpurun_out/hold/unet1024_h${h}_$i.log)"
  done
done
for i in 1 2; do
  for h in 1 0; do
    DLMPI_STREAM_HOLD=$h timeout -k 10 300 python bench.py --steps 20 --warmup 5 --mem 1 \
      > gpurun_out/hold/rn50_h${h}_$i.log 2>&1 || exit 1
    echo "rn50 hold=$h #$i $(grep -o '"value": [0-9.]*' gpurun_out/hold/rn50_h${h}_$i.log) $(grep -o 'peak_reserved_gb": [0-9.]*' gpurun_out/hold/rn50_h${h}_$i.log) $(grep -o 'peak_allocated_gb": [0-9.]*' gpurun_out/hold/rn50_h${h}_$i.log)"
  done
done
DLMPI_STREAM_HOLD=1 timeout -k 10 300 python bench.py --config unet512 --steps 10 --warmup 3 --mem 1 \
  > gpurun_out/hold/unet512_h1.log 2>&1 || exit 1
echo "unet512 hold=1 $(grep -o '"value": [0-9.]*' gpurun_out/hold/unet512_h1.log) $(grep -o 'peak_reserved_gb": [0-9.]*' gpurun_out/hold/unet512_h1.log)"
