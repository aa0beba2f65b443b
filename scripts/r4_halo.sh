#!/bin/bash
# Round 4: 256-pixel halo tiles against the 128-pixel ones and the pipelined 8-wave tiles on the
# stride-1 3x3 layers the halo path serves (conv lab, bitwise/stats check + timing), then one PMC pass
# per HALO_PMC spec.  Output: gpurun_out/r4_halo/
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4_halo${TAG:+_$TAG}; mkdir -p $O
cd $R
SH=${SHAPES:-"256,56,56,64,64,3,1,1 256,28,28,128,128,3,1,1 16,512,512,64,64,3,1,1 16,256,256,128,128,3,1,1 16,128,128,256,256,3,1,1 16,64,64,512,512,3,1,1"}
timeout -k 10 400 ./benchmarks/conv_lab 5 $SH > $O/lab.log 2>&1 || { echo lab failed; tail -5 $O/lab.log; exit 1; }
echo "lab OK=$(grep -c ' OK ' $O/lab.log) BAD=$(grep -c ' BAD ' $O/lab.log)"
cd /tmp && export TMPDIR=/tmp
CTR="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS"
i=0
for spec in ${HALO_PMC}; do
  v=${spec%%@*}; sh=${spec##*@}
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $CTR --kernel-trace -d $O/pmc$i -o c --output-format csv -- $R/benchmarks/conv_lab --only=$v 2 $sh > $O/pmc$i.log 2>&1
  rc=$?; echo "pmc$i $v $sh rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
