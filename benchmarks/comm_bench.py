"""RCCL collective benchmark over the framework's own communicator (csrc/binding/comm.cpp RcclComm):
all-reduce and broadcast bus bandwidth against message size (4 KB - 256 MB) at every channel cap in
``--caps`` (RCCL maxCTAs per communicator; 0 = RCCL's own choice), one JSON line per point on rank 0.

It is the instrument for the first N-GPU run: the gradient buckets (2 / 32 / 4 MB caps, parallel/ddp.py)
and the 16-channel default (parallel/comm.py DEFAULT_RCCL_CHANNELS) were chosen on a one-GPU comm-load
rehearsal with a MODELED 25 GB/s per channel (bench.py --rehearse); this measures the real curve.

    python benchmarks/comm_bench.py --gpus 8                  # starts 8 ranks itself (torchrun; --launcher mpirun)
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 benchmarks/comm_bench.py --gpus 8
    python benchmarks/comm_bench.py --gpus 1                  # world-1 RCCL (launch path / schema check)
    python benchmarks/comm_bench.py --gpus 2 --backend gloo   # CPU dry run of the multi-rank path (same schema)

Per point: {"op", "bytes", "n_ranks", "max_ctas", "time_us" (median of --iters, max over ranks),
"algbw_gbps", "busbw_gbps" (nccl-tests convention: all-reduce x 2 (n-1)/n), "backend"}.  A last line
{"summary": ...} gives per cap the peak bus bandwidth and the bandwidth at the bucket sizes.
Reference: the DDP gradient all-reduce of /root/reference/pytorch/unet/train.py:68-70 (NCCL), launched
N-wide by /root/reference/pytorch/unet/run.sh:100-112.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

BUCKET_MB = (2, 4, 32)   # parallel/ddp.py bucket caps (first / last / middle)


def sizes(lo: int, hi: int):
    """Powers of 4 from lo, plus the bucket caps, within [lo, hi]."""
    out, s = set(), lo
    while s <= hi:
        out.add(s)
        s *= 4
    out.update(mb << 20 for mb in BUCKET_MB if lo <= mb << 20 <= hi)
    return sorted(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--launcher", default="torchrun", choices=("torchrun", "mpirun"))
    ap.add_argument("--backend", default="rccl", choices=("rccl", "gloo"))
    ap.add_argument("--caps", default="8,16,32,0", help="channel caps (RCCL maxCTAs per communicator; 0: RCCL's)")
    ap.add_argument("--ops", default="allreduce,broadcast")
    ap.add_argument("--min_bytes", type=int, default=4 << 10)
    ap.add_argument("--max_bytes", type=int, default=256 << 20)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    args = ap.parse_args()
    import bench   # the launcher helpers (no torch import at module level)

    if args.gpus > 1 and not bench._under_launcher():
        sys.exit(bench.launch_ranks(args.gpus, args.launcher, sys.argv[1:], script=os.path.abspath(__file__)))

    import torch

    from deeplearning_mpi_amd.parallel.comm import bus_gbps, init_distributed, subcomm_uid, time_allreduce

    os.environ["DLMPI_RCCL_CHANNELS"] = "0"   # the bootstrap communicator: no process-wide cap
    os.environ.pop("NCCL_MAX_NCHANNELS", None)
    comm = init_distributed(args.backend)
    world, rank = comm.world_size, comm.rank
    if world != args.gpus:
        print(f"[comm_bench] world size {world} != --gpus {args.gpus}", file=sys.stderr, flush=True)
        sys.exit(2)
    dev = comm.device
    ops = [o for o in args.ops.split(",") if o]
    caps = [int(c) for c in args.caps.split(",") if c != ""]
    rows = []

    def emit(d):
        rows.append(d)
        if rank == 0:
            print(json.dumps(d), flush=True)

    if args.backend == "gloo":
        # CPU dry run: host-timed collectives of the torch gloo group, one "cap" (none)
        for op in ops:
            for nb in sizes(args.min_bytes, min(args.max_bytes, 16 << 20)):
                t = torch.ones(max(1, nb // 4), dtype=torch.float32)
                fn = (lambda: comm.allreduce(t)) if op == "allreduce" else (lambda: comm.broadcast(t, 0))
                for _ in range(args.warmup):
                    fn()
                ts = []
                for _ in range(args.iters):
                    a = time.perf_counter()
                    fn()
                    ts.append(time.perf_counter() - a)
                ts.sort()
                med = torch.tensor([ts[len(ts) // 2]], dtype=torch.float64)
                comm.allreduce(med, "max")
                sec = float(med)
                emit({"op": op, "bytes": nb, "n_ranks": world, "max_ctas": None, "time_us": round(sec * 1e6, 2),
                      "algbw_gbps": round(nb / sec / 1e9, 3), "busbw_gbps": round(bus_gbps(op, nb, sec, world), 3),
                      "backend": "gloo"})
    else:
        from deeplearning_mpi_amd._ext import native

        C = native()
        inner = getattr(comm, "inner", comm)
        base = getattr(inner, "c", None)
        if base is None:   # world size 1: init_distributed keeps no communicator; a world-1 RCCL one
            base = C.RcclComm(C.RcclComm.unique_id(), 0, 1, dev.index or 0)
        for cap in caps:
            nc = base if cap == 0 else C.RcclComm(subcomm_uid(base, rank, dev), rank, world, dev.index or 0, cap)
            for op in ops:
                for nb in sizes(args.min_bytes, args.max_bytes):
                    it = args.iters if nb <= (64 << 20) else max(5, args.iters // 4)
                    sec = time_allreduce(nc, nb, dev, iters=it, warmup=args.warmup, op=op)
                    emit({"op": op, "bytes": nb, "n_ranks": world, "max_ctas": cap,
                          "time_us": round(sec * 1e6, 2), "algbw_gbps": round(nb / sec / 1e9, 2),
                          "busbw_gbps": round(bus_gbps(op, nb, sec, world), 2), "backend": "rccl"})
            if nc is not base:
                nc.destroy()
        if base is not getattr(inner, "c", None):
            base.destroy()
    summary = {}
    for r in rows:
        key = f"{r['op']}@{r['max_ctas']}"
        s = summary.setdefault(key, {"peak_busbw_gbps": 0.0})
        s["peak_busbw_gbps"] = max(s["peak_busbw_gbps"], r["busbw_gbps"])
        for mb in BUCKET_MB:
            if r["bytes"] == mb << 20:
                s[f"busbw_gbps_at_{mb}MB"] = r["busbw_gbps"]
    if rank == 0:
        print(json.dumps({"summary": summary, "n_ranks": world, "backend": args.backend}), flush=True)
    from deeplearning_mpi_amd.parallel.comm import destroy_distributed

    destroy_distributed()


if __name__ == "__main__":
    main()
