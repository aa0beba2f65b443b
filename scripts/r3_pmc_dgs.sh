#!/bin/bash
# PMC counters of the layer-1 conv1 data gradient: streaming kernel vs the general kernel.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O="$R/gpurun_out/r3_pmc_dgs"; mkdir -p "$O"
for st in 1 0; do
  D="$O/stream$st"; mkdir -p "$D"; j=0
  for grp in "SQ_WAVES SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES" "FETCH_SIZE" "WRITE_SIZE"; do
    j=$((j+1))
    timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace -d "$D/pmc$j" -o c --output-format csv -- python3 "$R/benchmarks/dgrad_one.py" --stream $st --iters 3 > "$D/pmc$j.log" 2>&1
    rc=$?; echo "stream$st pmc$j rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$D/pmc$j.log"; exit $rc; }
  done
done
