#!/bin/bash
# Conv lab on the GPU box (benchmarks/conv_lab: every kernel variant on every shape, interleaved rounds,
# bitwise / statistics check), then one rocprofv3 --pmc pass (8 SQ counters) per PMC_SPECS entry
# "variant@N,H,W,C,K,R,stride,pad".  Build the lab first on the CPU side (benchmarks/conv_lab.cpp).
#   SHAPES="256,14,14,256,256,3,1,1 ..." ROUNDS=5 PMC_SPECS="pipe224x256v2@256,14,14,256,256,3,1,1" TAG=x
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/lab${TAG:+_$TAG}; mkdir -p $O
cd $R
timeout -k 10 400 ./benchmarks/conv_lab ${ROUNDS:-5} ${SHAPES} > $O/lab.log 2>&1 || { echo lab failed; tail -5 $O/lab.log; exit 1; }
echo "lab OK=$(grep -c ' OK ' $O/lab.log) BAD=$(grep -c ' BAD ' $O/lab.log)"
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
