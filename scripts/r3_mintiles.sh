#!/bin/bash
# A/B of the 256-row tile floor (DLMPI_CONV_BM256_MIN_TILES 256 default vs 192): ResNet-152 at bs 128
# has 196-tile 14^2 grids.  Output: gpurun_out/r3_mintiles/
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && export HSA_ENABLE_IPC_MODE_LEGACY=0
O="$R/gpurun_out/r3_mintiles"; mkdir -p "$O"
for i in 1 2; do for v in 256 192; do for c in resnet152 resnet50 unet512; do
  DLMPI_CONV_BM256_MIN_TILES=$v timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 > "$O/${c}_${v}_$i.log" 2>&1 || { echo "bench $c $v failed"; tail -5 "$O/${c}_${v}_$i.log"; exit 1; }
  echo "$c $v $i $(grep -o '"value": [0-9.]*' $O/${c}_${v}_$i.log)"
done; done; done
