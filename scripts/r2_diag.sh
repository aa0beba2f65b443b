#!/bin/bash
# Conv-kernel diagnostics on one box: per-shape ResNet-50 conv table (ours vs MIOpen), hipBLASLt
# ceiling of the same GEMMs, 1x1 memory roofline, and PMC counter groups of the short-reduction
# expand 1x1 forward (56^2 64->256) and the 14^2 3x3.  Output: gpurun_out/r2_diag/
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && export HSA_ENABLE_IPC_MODE_LEGACY=0
O="$R/gpurun_out/r2_diag"; mkdir -p "$O"
timeout -k 10 400 python benchmarks/conv_bench.py --net resnet50 --iters 20 > "$O/conv_bench_r50.log" 2>&1 || { echo "conv_bench failed"; tail -5 "$O/conv_bench_r50.log"; exit 1; }
tail -1 "$O/conv_bench_r50.log"
timeout -k 10 300 python benchmarks/gemm_ceiling.py --iters 20 > "$O/gemm_ceiling.log" 2>&1 || { echo "gemm_ceiling failed"; tail -5 "$O/gemm_ceiling.log"; exit 1; }
timeout -k 10 300 python benchmarks/conv_roofline.py --iters 20 > "$O/roofline.log" 2>&1 || { echo "roofline failed"; tail -5 "$O/roofline.log"; exit 1; }
cd /tmp && export TMPDIR=/tmp
i=0
for shp in "256,56,56,64,256,1,1,0" "256,14,14,256,256,3,1,1"; do for grp in "SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVES" "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum" "SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace -d "$O/pmc$i" -o c --output-format csv -- python3 "$R/benchmarks/conv_one.py" --shape $shp --pass fwd --iters 5 > "$O/pmc$i.log" 2>&1
  rc=$?; echo "pmc$i rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$O/pmc$i.log"; exit $rc; }
done; done
echo done
