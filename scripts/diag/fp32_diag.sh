#!/bin/bash
# fp32 UNet gradient error under several kernel-path knobs (one process each)
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/diag
mkdir -p $O
run() { tag=$1; shift; env "$@" timeout -k 10 200 python scripts/diag/fp32_unet_diag.py > $O/$tag.log 2>&1 || { echo "$tag failed"; tail -5 $O/$tag.log; exit 1; }; echo "$tag: $(grep -c '<<<' $O/$tag.log) bad, first: $(grep -m1 '<<<' $O/$tag.log | tr -s ' ')"; }
run a1 X=1
run a2 X=1
run nofin DLMPI_BN_FUSED_FINALIZE=0
run nofuse DLMPI_FUSE_BN_BWD=0
run nosplit DLMPI_CONV_SPLITK=0
run nosplit2 DLMPI_CONV_SPLITK=0
run fence DLMPI_FIN_SC1=0
run nostreams DLMPI_WGRAD_STREAM=0 DLMPI_BRANCH_STREAM=0
