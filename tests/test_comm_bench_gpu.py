"""RCCL instruments for the first N-GPU run, on one GPU (world-size-1 RCCL; the N-rank curve is the
driver's): per-communicator channel caps (ncclCommInitRankConfig maxCTAs), sub-communicators over a
broadcast id, the auto-cap calibration, the collective benchmark's JSON, and bench.py's per-bucket
comm-stream timing (dist.bucket_probe)."""
import json
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _native():
    from deeplearning_mpi_amd._ext import native

    return native()


def test_capped_communicator_and_subcomm():
    from deeplearning_mpi_amd.parallel.comm import calibrate_channels, subcomm_uid

    C = _native()
    dev = torch.device("cuda", torch.cuda.current_device())
    base = C.RcclComm(C.RcclComm.unique_id(), 0, 1, dev.index)
    sub = C.RcclComm(subcomm_uid(base, 0, dev), 0, 1, dev.index, 8)
    assert base.max_ctas() == 0 and sub.max_ctas() == 8
    t = torch.arange(1 << 20, dtype=torch.float32, device=dev)
    ref = t.clone()
    sub.allreduce(t, "sum", False)
    torch.cuda.synchronize()
    assert torch.equal(t, ref)   # world size 1: the identity, through the capped communicator
    cal = calibrate_channels(base, 0, 1, dev, nbytes=4 << 20, iters=3)
    assert [r["max_ctas"] for r in cal["rows"]] == [0, 8, 16, 32] and cal["chosen"] == 0
    sub.destroy()
    base.destroy()


def test_comm_bench_world1_schema():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "benchmarks", "comm_bench.py"), "--gpus", "1",
                        "--max_bytes", str(4 << 20), "--iters", "3", "--warmup", "1"],
                       cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    pts = [l for l in lines if "op" in l]
    assert {p["max_ctas"] for p in pts} == {8, 16, 32, 0}
    assert all(p["backend"] == "rccl" and p["time_us"] > 0 and p["algbw_gbps"] > 0 for p in pts)
    assert "summary" in lines[-1]


def test_bench_rccl1_bucket_probe():
    r = subprocess.run([sys.executable, "bench.py", "--config", "resnet18_cifar", "--steps", "2", "--warmup", "1",
                        "--rccl1", "1", "--graph", "0"], cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    (j,) = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{") and '"metric"' in l]
    d = j["dist"]
    bp = d["bucket_probe"]
    assert bp is not None and len(bp["buckets"]) == len(d["bucket_mb"])
    for b in bp["buckets"]:
        assert b["dur_ms"] >= 0 and b["start_ms"] >= 0
    assert bp["backward_compute_end_ms"] > 0 and "comm_tail_ms" in bp
