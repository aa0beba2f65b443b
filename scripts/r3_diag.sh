#!/bin/bash
# Round-3 triage of the GPU-suite failures after the autotuner commit + autotune A/B.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3_diag; mkdir -p $O
cat > $O/wd_child.py <<'PY'
import sys, torch
from deeplearning_mpi_amd._ext import native
C = native()
torch.cuda.set_device(0)
c = C.RcclComm(C.RcclComm.unique_id(), 0, 1, 0)
t = torch.ones(1024, device="cuda")
c.allreduce(t, "sum", False)
torch.cuda.synchronize()
print("completed", float(t[0]), flush=True)
if sys.argv[1] == "destroy":
    c.destroy()
elif sys.argv[1] == "del":
    del c
print("end", flush=True)
PY
for m in none destroy del; do
  PYTHONPATH=$R timeout -k 5 60 python $O/wd_child.py $m > $O/wd_$m.log 2>&1; echo "wd $m rc=$?"
done
DLMPI_CONV_AUTOTUNE=0 timeout -k 10 400 python -u -m pytest -q --timeout 180 --timeout-method thread tests/test_fp32_gpu.py tests/test_dual_dgrad_gpu.py tests/test_apps_gpu.py > $O/at0_tests.log 2>&1; echo "at0 tests rc=$?"; tail -3 $O/at0_tests.log
CONFIGS="resnet50" STEPS=20 REPS=2 VARIANTS='base at0=DLMPI_CONV_AUTOTUNE=0' bash scripts/env_ab3.sh
