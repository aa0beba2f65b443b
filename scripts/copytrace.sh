#!/bin/bash
# Where do the step's D2D copies / ATen kernels come from: rocprofv3 HIP-API + kernel trace of a short
# bench.py run, then scripts/copytrace.py pairs every hipMemcpy* / ATen launch with its neighbours.
#   CONFIGS="resnet50 unet512" TAG=x bash scripts/copytrace.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/copytrace${TAG:+_$TAG}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
for c in ${CONFIGS:-resnet50}; do
  timeout -k 10 240 rocprofv3 --hip-trace --kernel-trace -d $O/$c -o t --output-format csv -- python3 $R/bench.py --config $c --steps 2 --warmup 2 --graph 0 > $O/$c.log 2>&1
  rc=$?; echo "$c rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/$c.log; exit $rc; }
  python3 $R/scripts/copytrace.py $O/$c > $O/${c}_copies.txt 2>&1; head -60 $O/${c}_copies.txt
done
exit 0
