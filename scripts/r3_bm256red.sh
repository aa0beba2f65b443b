#!/bin/bash
# A/B of the 256-row tile for 1x1 convs with reduction >= 1024 (DLMPI_CONV_BM256_MIN_RED_1X1 1024
# default vs 2304 = round-3 baseline): the 14^2 1024->256 forward / 256<-1024 data gradient.
# ResNet-50 and ResNet-152 (bs 128: its 14^2 grids stay below the 256-tile floor) bench pairs.
# Output: gpurun_out/r3_bm256red2/
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && export HSA_ENABLE_IPC_MODE_LEGACY=0
O="$R/gpurun_out/r3_bm256red2"; mkdir -p "$O"
for i in 1 2; do for v in 2304 1024; do for c in resnet50 resnet152; do
  DLMPI_CONV_BM256_MIN_RED_1X1=$v timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 > "$O/${c}_${v}_$i.log" 2>&1 || { echo "bench $c $v failed"; tail -5 "$O/${c}_${v}_$i.log"; exit 1; }
  echo "$c $v $i $(grep -o '"value": [0-9.]*' $O/${c}_${v}_$i.log)"
done; done; done
