#!/bin/bash
# PMC counters of the weight-gradient kernel on the shapes that dominate ResNet-50 / UNet wgrad time.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O="$R/gpurun_out/pmc_wgrad"; mkdir -p "$O"
for shp in ${SHAPES:-"256,56,56,64,64,3,1,1" "16,512,512,64,64,3,1,1" "16,256,256,128,128,3,1,1" "256,14,14,1024,256,1,1,0"}; do
  timeout -k 5 120 python "$R/benchmarks/conv_one.py" --shape $shp --pass wgrad --iters 10 >> "$O/times.log" 2>&1 || { echo "time $shp failed"; exit 1; }
  j=0; D="$O/$(echo $shp | tr ',' '_')"; mkdir -p "$D"
  for grp in "SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD SQ_WAVES SQ_INSTS_SALU" "SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU" "FETCH_SIZE"; do
    j=$((j+1))
    timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace -d "$D/pmc$j" -o c --output-format csv -- python3 "$R/benchmarks/conv_one.py" --shape $shp --pass wgrad --iters 3 > "$D/pmc$j.log" 2>&1
    rc=$?; echo "pmc$j $shp rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$D/pmc$j.log"; exit $rc; }
  done
done
cat "$O/times.log"
