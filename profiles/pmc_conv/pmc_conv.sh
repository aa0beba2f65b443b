#!/bin/bash
# PMC counters for representative conv kernels (one kernel per run; counters in small groups).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p "$R/gpurun_out/pmc"
i=0
for spec in "16,64,64,512,512,3,1,1 fwd" "256,56,56,64,256,1,1,0 fwd" "256,14,14,256,256,3,1,1 wgrad" "256,28,28,128,128,3,1,1 fwd"; do
  set -- $spec
  for grp in "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS" "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_INSTS_MFMA" "SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU"; do
    i=$((i+1))
    timeout -k 10 120 rocprofv3 --pmc $grp --kernel-trace -d "$R/gpurun_out/pmc/run$i" -o c --output-format csv -- python "$R/benchmarks/conv_one.py" --shape $1 --pass $2 --iters 5 > "$R/gpurun_out/pmc/run$i.log" 2>&1
    rc=$?; echo "run$i $1 $2 rc=$rc"; [ $rc -ne 0 ] && exit $rc
  done
done
