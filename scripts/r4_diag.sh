#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/diag
PYTHONPATH=$R timeout -k 10 300 python scripts/diag/apply_bw.py > gpurun_out/diag/apply_bw.log 2>&1 || { echo apply_bw failed; tail -3 gpurun_out/diag/apply_bw.log; exit 1; }
grep -v Warn gpurun_out/diag/apply_bw.log
cd /tmp && export TMPDIR=/tmp
PYTHONPATH=$R timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/diag/which -o w -- python3 $R/scripts/diag/which_kernel.py > $R/gpurun_out/diag/which.log 2>&1 || { echo which failed; tail -3 $R/gpurun_out/diag/which.log; exit 1; }
echo which done
