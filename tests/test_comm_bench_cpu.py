"""The collective benchmark (benchmarks/comm_bench.py) and the channel-cap calibration rule
(parallel/comm.py choose_cap / bus_gbps): the JSON schema of a 2-rank gloo dry run of the same
multi-rank path the N-GPU RCCL run takes, and the cap choice on synthetic measurements."""
import json
import os
import subprocess
import sys

import pytest

from deeplearning_mpi_amd.parallel.comm import AUTO_CAPS, bus_gbps, choose_cap

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bus_bandwidth_convention():
    # nccl-tests: all-reduce bus bandwidth = algbw * 2 (n-1)/n, broadcast = algbw
    assert bus_gbps("allreduce", 8e9, 1.0, 8) == pytest.approx(8 * 2 * 7 / 8)
    assert bus_gbps("broadcast", 8e9, 1.0, 8) == pytest.approx(8.0)
    assert bus_gbps("allreduce", 8e9, 1.0, 1) == 0.0


def test_choose_cap_smallest_within_fraction():
    rows = [{"max_ctas": 0, "busbw_gbps": 300.0}, {"max_ctas": 8, "busbw_gbps": 180.0},
            {"max_ctas": 16, "busbw_gbps": 285.0}, {"max_ctas": 32, "busbw_gbps": 310.0}]
    assert choose_cap(rows, 8) == 16          # 285 >= 0.9 * 310; 8 is not
    assert choose_cap(rows, 1) == 0           # no bus at world size 1
    assert choose_cap([{"max_ctas": 0, "busbw_gbps": 300.0}, {"max_ctas": 8, "busbw_gbps": 100.0}], 8) == 0
    assert set(AUTO_CAPS) == {8, 16, 32}


def test_comm_bench_gloo_two_ranks_schema():
    env = dict(os.environ, PYTHONPATH=ROOT)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "benchmarks", "comm_bench.py"), "--gpus", "2",
                          "--backend", "gloo", "--max_bytes", str(4 << 20), "--iters", "2", "--warmup", "1"],
                         stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=300, env=env, cwd="/tmp")
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [json.loads(l) for l in out.stdout.splitlines() if l.startswith("{")]
    pts = [l for l in lines if "op" in l]
    summ = [l for l in lines if "summary" in l]
    assert len(summ) == 1 and summ[0]["n_ranks"] == 2
    assert {p["op"] for p in pts} == {"allreduce", "broadcast"}
    for p in pts:
        assert set(p) == {"op", "bytes", "n_ranks", "max_ctas", "time_us", "algbw_gbps", "busbw_gbps", "backend"}
        assert p["n_ranks"] == 2 and p["time_us"] > 0 and p["busbw_gbps"] > 0
    sizes = sorted({p["bytes"] for p in pts})
    assert sizes[0] == 4 << 10 and (2 << 20) in sizes and (4 << 20) in sizes   # the bucket caps are points
    assert "busbw_gbps_at_2MB" in summ[0]["summary"]["allreduce@None"]
