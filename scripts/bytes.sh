#!/bin/bash
# HBM traffic per kernel of a training step: two rocprofv3 --pmc passes over a short bench.py run
# (FETCH_SIZE, WRITE_SIZE: KB per dispatch; dispatches are serialized under --pmc), then
# scripts/bytes_digest.py.   CONFIGS="resnet50 unet512" TAG=x bash scripts/bytes.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/bytes${TAG:+_$TAG}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
for c in ${CONFIGS:-resnet50}; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 240 rocprofv3 --pmc $ctr --kernel-trace -d $O/${c}_$ctr -o c --output-format csv -- python3 $R/bench.py --config $c --steps ${STEPS:-2} --warmup 1 --graph 0 > $O/${c}_$ctr.log 2>&1
    rc=$?; echo "$c $ctr rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/${c}_$ctr.log; exit $rc; }
  done
  python3 $R/scripts/bytes_digest.py $O/${c}_FETCH_SIZE $O/${c}_WRITE_SIZE --steps $((${STEPS:-2} + 1)) > $O/${c}_bytes.md
  head -40 $O/${c}_bytes.md
done
exit 0
