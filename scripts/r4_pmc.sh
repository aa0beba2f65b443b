#!/bin/bash
# One PMC pass (8 SQ counters) per conv_lab variant@shape in PMC_SPECS.  Output: gpurun_out/r4_pmc/
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4_pmc${TAG:+_$TAG}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
CTR=${CTR:-"SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS"}
i=0
for spec in ${PMC_SPECS}; do
  v=${spec%%@*}; sh=${spec##*@}
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $CTR --kernel-trace -d $O/pmc$i -o c --output-format csv -- $R/benchmarks/conv_lab --only=$v 2 $sh > $O/pmc$i.log 2>&1
  rc=$?; echo "pmc$i $v $sh rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
