#!/bin/bash
# PMC counters of the 3x3 weight gradient (one kernel, one counter group per run) for each
# set_wgrad3_variant in ${VARIANTS} on shape ${SHAPE}.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out/pmc_w3; mkdir -p $O
SHAPE=${SHAPE:-16,64,64,1536,512,3,1,1}
i=0
for v in ${VARIANTS:-0 18}; do
  for grp in "SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS" \
             "SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_SALU TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace -d $O/pmc$i -o c --output-format csv -- python $R/benchmarks/conv_one.py --shape $SHAPE --pass wgrad --iters 5 --set set_wgrad3_variant=$v > $O/run$i.log 2>&1
    rc=$?; echo "run$i v=$v rc=$rc"; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
