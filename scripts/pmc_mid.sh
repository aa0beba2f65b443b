#!/bin/bash
# PMC counters of the ResNet-50 layer-1 expand 1x1 forward (our conv kernel), one counter group per run
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O="$R/gpurun_out/pmc_mid"; mkdir -p "$O"
i=0
for shp in "256,14,14,1024,256,1,1,0" "256,14,14,256,256,3,1,1"; do for grp in "SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVES" "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum" "SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace -d "$O/run$i" -o c --output-format csv -- python "$R/benchmarks/conv_one.py" --shape $shp --pass fwd --iters 5 > "$O/run$i.log" 2>&1
  rc=$?; echo "run$i rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$O/run$i.log"; exit $rc; }
done; done
