#!/bin/bash
# PMC counters of one conv pass (benchmarks/conv_one.py) per extension-setter variant: two counter
# groups per variant, one rocprofv3 run per group.  SHAPE, PASS, SETS="a=1,b=0 a=0" (space-separated).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out/pmc_conv${TAG:+_$TAG}; mkdir -p $O
SHAPE=${SHAPE:-16,64,64,512,512,3,1,1}
i=0
for v in ${SETS:-none}; do
  set_arg=""; [ "$v" != "none" ] && set_arg="--set $v"
  for grp in "SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS" \
             "SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_SALU TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace -d $O/pmc$i -o c --output-format csv -- python $R/benchmarks/conv_one.py --shape $SHAPE --pass ${PASS:-fwd} --iters 5 $set_arg > $O/run$i.log 2>&1
    rc=$?; echo "run$i $v rc=$rc"; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
