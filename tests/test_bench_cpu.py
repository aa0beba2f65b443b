"""bench.py's launch contract on CPU (gloo dry run of the multi-rank path):

* ``--gpus N`` without a launcher environment starts N ranks itself (torchrun or mpirun) and rank 0
  prints ONE JSON line with ``n_gpus: N``;
* under a launcher, ``--gpus`` must equal the world size (exit code 2 otherwise) -- the round-1
  harness silently measured one rank when asked for eight (missing item 1).
"""
import json
import os
import shutil
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SMALL = ["--backend", "gloo", "--config", "resnet18_cifar", "--batch", "4", "--steps", "2", "--warmup", "1"]


def _env():
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "PMI_RANK", "PMI_SIZE",
              "OMPI_COMM_WORLD_RANK"):
        env.pop(k, None)
    return env


def _json_lines(out):
    return [json.loads(l) for l in out.splitlines() if l.startswith("{")]


@pytest.mark.parametrize("launcher", ["torchrun", "mpirun"])
def test_bench_self_launches_n_ranks(launcher):
    if launcher == "mpirun" and not (shutil.which("mpirun") or os.path.exists("/opt/conda/bin/mpirun")):
        pytest.skip("no mpirun")
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--launcher", launcher, *SMALL], cwd=ROOT,
                       env=_env(), capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout   # rank 0 only
    j = lines[0]
    assert j["n_gpus"] == 2 and j["config"]["parallelism"] == "dp2" and j["config"]["global_batch"] == 8
    assert j["steps"] == 2 and j["warmup"] == 1 and j["value"] > 0
    # distributed facts: bucket layout, per-rank step times, exposed all-reduce
    d = j["dist"]
    assert d["reducer"] and len(d["bucket_mb"]) >= 1 and d["comm_exposed_ms"] is not None
    assert 0 < d["per_rank_ms_per_step"]["min"] <= d["per_rank_ms_per_step"]["max"]
    assert d["per_rank_ms_per_step"]["max"] == pytest.approx(j["ms_per_step"], rel=1e-3, abs=1e-3)
    # the RCCL-only instruments are reported (empty on gloo): per-bucket comm-stream timing, channel calibration
    assert "bucket_probe" in d and "rccl_channel_calibration" in d


def test_bench_single_rank_unchanged():
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "1", *SMALL], cwd=ROOT, env=_env(),
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    (j,) = _json_lines(r.stdout)
    assert j["n_gpus"] == 1 and j["config"]["parallelism"] == "dp1"


def test_bench_rejects_world_size_mismatch():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nproc-per-node", "2", "--master-addr",
                        "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "4", *SMALL], cwd=ROOT,
                       env=_env(), capture_output=True, text=True, timeout=600)
    assert r.returncode != 0
    assert "--gpus 4 but the launcher started 2 ranks" in r.stderr


def test_bench_kernel_pins_parse():
    """--pin (A/B only) sets the extension's kernel-choice switches by name and runs the step."""
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "1", "--pin", "pipe=0,halo=0,wgrad_batch=8,defer=0",
                        *SMALL], cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    (j,) = _json_lines(r.stdout)
    assert j["n_gpus"] == 1
