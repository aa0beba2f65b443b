#!/bin/bash
# Weight-gradient lab on the GPU box (benchmarks/wgrad_lab.py), optional GPU tests first.
#   ARMS="new:;old:set_wgrad3_var=0" LABARGS="--only3x3" TESTK="wgrad" TAG=x bash scripts/wlab.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && export HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out/wlab${TAG:+_$TAG}; mkdir -p $O
if [ -n "$TESTK" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -k "$TESTK" > $O/tests.log 2>&1
  rc=$?; tail -1 $O/tests.log
  if [ $rc -ne 0 ]; then grep -E "^FAILED|^ERROR|Error" $O/tests.log | head -20; exit 1; fi
fi
timeout -k 10 ${LABTIME:-600} python -u benchmarks/wgrad_lab.py --arms "${ARMS:-base:}" ${LABARGS} > $O/lab.log 2>&1
rc=$?; cat $O/lab.log | tail -40; [ $rc -ne 0 ] && exit $rc
# PMC passes: PMC_SPECS="shape@setters ..." (conv_one.py --pass wgrad), one 8-SQ-counter run each
cd /tmp && export TMPDIR=/tmp
CTR=${CTR:-"SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS"}
i=0
for spec in ${PMC_SPECS}; do
  sh=${spec%%@*}; st=${spec#*@}; [ "$st" = "$spec" ] && st=""
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $CTR --kernel-trace -d $O/pmc$i -o c --output-format csv -- python3 $R/benchmarks/conv_one.py --shape $sh --pass wgrad --iters 5 --set "$st" > $O/pmc$i.log 2>&1
  rc=$?; echo "pmc$i $sh $st rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
