"""Failure detection on the GPU data plane: a collective that does not complete
within DLMPI_COMM_TIMEOUT makes the RCCL watchdog abort the communicator and end the process with
exit code 70 (instead of hanging the job).  The "hang" is injected with a bounded delay kernel
(DLMPI_FAULT_COMM_DELAY_MS, always finishes) queued in front of the all-reduce."""
import os
import subprocess
import sys
import time

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import torch
from deeplearning_mpi_amd._ext import native
C = native()
torch.cuda.set_device(0)
c = C.RcclComm(C.RcclComm.unique_id(), 0, 1, 0)
t = torch.ones(1024, device="cuda")
c.allreduce(t, "sum", False)
torch.cuda.synchronize()
print("completed", float(t[0]))
"""


def _run(env_extra, timeout=120):
    env = dict(os.environ, PYTHONPATH=ROOT, **env_extra)
    t0 = time.time()
    r = subprocess.run([sys.executable, "-c", CHILD], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=timeout)
    return r, time.time() - t0


def test_watchdog_aborts_stuck_collective():
    r, dt = _run({"DLMPI_COMM_TIMEOUT": "1.5", "DLMPI_FAULT_COMM_DELAY_MS": "6000"})
    assert r.returncode == 70, (r.returncode, r.stdout, r.stderr)
    assert "[dlmpi watchdog]" in r.stderr and "allreduce" in r.stderr


def test_watchdog_quiet_on_healthy_collective():
    r, _ = _run({"DLMPI_COMM_TIMEOUT": "30", "DLMPI_FAULT_COMM_DELAY_MS": "300"})
    assert r.returncode == 0, r.stderr
    assert "completed 1.0" in r.stdout
