"""Benchmark harness: DDP training throughput, images/sec for the whole job.

Default = the headline config of BASELINE.json: ResNet-50, bs=256 per GPU, 3x224x224 synthetic
ImageNet-shaped data, random-init weights, bf16 compute (fp32 master weights, fp32 gradient
all-reduce), SGD momentum 0.9 / wd 1e-5 (the reference optimizer,
/root/reference/pytorch/resnet/main.py:114), one process per GPU over RCCL.  Every timed step is
a full training step: forward, loss, backward with bucketed gradient all-reduce, optimizer update.

The other BASELINE.json configs are presets (``--config``):
  resnet50        ResNet-50  bs=256/GPU 3x224x224, SGD, CE            (headline, default)
  resnet152       ResNet-152 bs=128/GPU 3x224x224, SGD, CE            (config 4)
  unet512         UNet bs=16/GPU 3x512x512 binary masks, Adam + BCE + clip 1.0  (config 3;
                  /root/reference/pytorch/unet/train.py:160-194, batch default :319)
  unet1024        UNet in_channels=1 bs=16/GPU 1x1024x1024, Adam + BCE + clip  (config 5)
  resnet18_cifar  ResNet-18 bs=128/GPU 3x32x32, 10 classes (the reference's own CIFAR run,
                  /root/reference/pytorch/resnet/main.py:36-54,164)

Usage:  python bench.py [--gpus N] [--steps K] [--warmup W] [--config NAME] [--graph 1] [--breakdown N]

Launch: one rank per GPU.  Under torch.distributed.run / torchrun or mpirun the ranks come from the
launcher's environment and ``--gpus`` must equal the world size (checked; a mismatch exits 2).
Without a launcher environment and N > 1, this process starts the N ranks itself BEFORE importing
torch or touching a GPU (``--launcher torchrun`` (default) or ``mpirun``, rendezvous at 127.0.0.1,
``HSA_ENABLE_IPC_MODE_LEGACY=0`` exported for dmabuf-only hosts), waits for them and exits with the
first non-zero return code -- the reference's launcher likewise spawns ``nproc_per_node`` workers
itself (/root/reference/pytorch/unet/run.sh:100-112).  ``--backend gloo`` is a CPU dry run of the
same multi-rank path (gloo all-reduce, CPU reference backend).
Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import socket
import subprocess
import sys
import time

# multi-process RCCL on dmabuf-only hosts (read by the HSA runtime at its first use, which is later)
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

BASELINE_VALUE = None   # the reference publishes no number

PRESETS = {
    "resnet50": dict(task="cls", arch="resnet50", batch=256, image=224, classes=1000, cin=3,
                     metric="images/sec (whole node) ResNet-50 DDP bs=256/GPU"),
    "resnet152": dict(task="cls", arch="resnet152", batch=128, image=224, classes=1000, cin=3,
                      metric="images/sec (whole node) ResNet-152 DDP bs=128/GPU"),
    "resnet18_cifar": dict(task="cls", arch="resnet18", batch=128, image=32, classes=10, cin=3,
                           metric="images/sec (whole node) ResNet-18 CIFAR-10 DDP bs=128/GPU"),
    "unet512": dict(task="seg", arch="unet", batch=16, image=512, classes=1, cin=3,
                    metric="images/sec (whole node) UNet-2D 3x512x512 DDP bs=16/GPU"),
    "unet1024": dict(task="seg", arch="unet", batch=16, image=1024, classes=1, cin=1,
                     metric="images/sec (whole node) UNet-2D 1x1024x1024 DDP bs=16/GPU"),
}


_LAUNCH_ENV = ("RANK", "WORLD_SIZE", "OMPI_COMM_WORLD_RANK", "PMI_RANK", "PMIX_RANK", "MV2_COMM_WORLD_RANK")


def _under_launcher() -> bool:
    return any(os.environ.get(k) not in (None, "") for k in _LAUNCH_ENV)


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int, launcher: str, argv, script: str | None = None) -> int:
    """Start ``n`` ranks of ``script`` (default: this one) as child processes (no torch import, no GPU
    touched in this process) and return the first non-zero exit code (0 if all ranks succeeded)."""
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", MASTER_ADDR="127.0.0.1")
    env["PYTHONPATH"] = ROOT + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
    script = script or os.path.abspath(__file__)
    if launcher == "mpirun":
        mpirun = shutil.which("mpirun") or "/opt/conda/bin/mpirun"
        cmd = [mpirun, "-n", str(n), sys.executable, script, *argv]
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(n),
               "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), script, *argv]
    print(f"[bench] launching {n} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
    return subprocess.call(cmd, env=env)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="resnet50", choices=sorted(PRESETS))
    ap.add_argument("--arch", default=None, help="override the preset's model")
    ap.add_argument("--batch", type=int, default=None, help="per-GPU batch (override)")
    ap.add_argument("--image", type=int, default=None)
    ap.add_argument("--classes", type=int, default=None)
    ap.add_argument("--bucket_mb", type=float, default=None)
    ap.add_argument("--graph", default="auto", choices=["auto", "0", "1"],
                    help="1: replay the whole step from a captured hipGraph; auto (default): the training app's "
                         "decision (apps/classification.py use_graph: on for launch-bound steps, e.g. the "
                         "reference's ResNet-18 on CIFAR; off where concurrent streams win)")
    ap.add_argument("--breakdown", type=int, default=0,
                    help="N > 0: after the timed steps, N more steps with HIP-event phase timing (forward / "
                         "backward / exposed all-reduce wait / optimizer), printed to stderr")
    ap.add_argument("--mem", type=int, default=0, help="1: print caching-allocator statistics (peak allocated / "
                                                       "reserved GB, allocation retries) to stderr")
    ap.add_argument("--backend", default="rccl", help="rccl (default); gloo: CPU dry run of the multi-rank path "
                                                      "(gloo + DLMPI_GLOO_DEVICE=cuda rehearses several ranks on one GPU)")
    ap.add_argument("--launcher", default="torchrun", choices=("torchrun", "mpirun"),
                    help="how --gpus N > 1 starts its ranks when not already under a launcher")
    ap.add_argument("--rccl1", type=int, default=0,
                    help="1 (single GPU only): run the step through a world-size-1 RCCL communicator with the "
                         "bucketed reducer forced on (every all-reduce / the K5 broadcast go through RCCL)")
    ap.add_argument("--rehearse", type=int, default=0,
                    help="C > 0 (single GPU): comm-load rehearsal of a --rehearse_world-rank all-reduce -- the "
                         "--rccl1 path plus, after every bucket all-reduce, C workgroups on the comm stream that "
                         "move the ring all-reduce's traffic and hold their CUs for the modeled collective time "
                         "(RCCL channels = C; parallel/comm.py rccl_channel_budget)")
    ap.add_argument("--rehearse_world", type=int, default=8)
    ap.add_argument("--rehearse_gbps_ch", type=float, default=25.0, help="modeled bus bandwidth per channel (GB/s)")
    ap.add_argument("--rehearse_gbps_max", type=float, default=400.0, help="modeled bus bandwidth cap (GB/s)")
    ap.add_argument("--rehearse_lds", type=int, default=32768, help="LDS bytes per modeled channel workgroup")
    ap.add_argument("--rehearse_lat_us", type=float, default=20.0, help="modeled latency per all-reduce (us)")
    ap.add_argument("--pyprof", type=int, default=0,
                    help="N > 0: after the timed steps, run N more steps under cProfile and print the top host "
                         "functions (self time) to stderr -- where the eager step's issue time goes")
    ap.add_argument("--host_time", type=int, default=0,
                    help="N > 0: after the timed steps, N more steps timing the HOST issue time of each step "
                         "(call to return, GPU running behind) against the GPU step time; printed to stderr")
    ap.add_argument("--pin", default="",
                    help="A/B only: kernel-choice pins NAME=V[,NAME=V] -- pipe / halo / stream / dgrad_stream / "
                         "autotune / wgrad3 / splitk (the extension's test setters; -1 = production choice), "
                         "defer=0 (weight-gradient reductions launched one by one)")
    ap.add_argument("--rccl_channels", default=None,
                    help="RCCL channel (CU) cap: N, 0 (RCCL's choice) or auto (calibrated at init: the smallest cap "
                         "of 8/16/32 reaching 90 %% of the best all-reduce bus bandwidth, parallel/comm.py "
                         "calibrate_channels); default DLMPI_RCCL_CHANNELS or 16")
    ap.add_argument("--precision", default="bf16", choices=["bf16", "fp32"],
                    help="compute precision of the native engine: bf16 (default, the BASELINE dtype) or fp32 "
                         "(the same kernels on fp32 storage -- how the reference trains ResNet-18 on CIFAR)")
    ap.add_argument("--bucket_probe", type=int, default=1,
                    help="1 (default): with an RCCL reducer (N > 1 or --rccl1) and no hipGraph, one untimed step "
                         "after the timed region times every bucket all-reduce on the comm stream (dist.buckets)")
    args = ap.parse_args()
    if args.rccl_channels is not None:
        os.environ["DLMPI_RCCL_CHANNELS"] = str(args.rccl_channels)
        os.environ.pop("NCCL_MAX_NCHANNELS", None)
    if args.rehearse > 0:
        args.rccl1 = 1
        os.environ["DLMPI_RCCL_CHANNELS"] = str(args.rehearse)
        os.environ.pop("NCCL_MAX_NCHANNELS", None)
    if args.gpus > 1 and not _under_launcher():
        sys.exit(launch_ranks(args.gpus, args.launcher, sys.argv[1:]))
    cfg = dict(PRESETS[args.config])
    for k in ("arch", "batch", "image", "classes"):
        if getattr(args, k) is not None:
            cfg[k] = getattr(args, k)

    import torch

    import deeplearning_mpi_amd as dl
    from deeplearning_mpi_amd.data import device_batch
    from deeplearning_mpi_amd.models import ARCHS, UNet
    from deeplearning_mpi_amd.ops import BCEWithLogitsLoss, CrossEntropyLoss, backward
    from deeplearning_mpi_amd.optim import SGD, Adam, clip_grad_norm_

    comm = dl.init_distributed(args.backend)
    world = comm.world_size
    dev = comm.device
    if world != args.gpus:
        print(f"[bench] --gpus {args.gpus} but the launcher started {world} ranks", file=sys.stderr, flush=True)
        sys.exit(2)
    if world > 1 and args.backend in ("rccl", "nccl") and "rccl" not in comm.backend:
        print(f"[bench] expected the RCCL data plane, got {comm.backend}", file=sys.stderr, flush=True)
        sys.exit(2)

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize()
    pins = dict(kv.split("=") for kv in args.pin.split(",") if kv)
    if pins:
        from deeplearning_mpi_amd._ext import native as _nat

        setters = {"pipe": "set_conv_pipe", "halo": "set_conv_halo", "stream": "set_conv_stream",
                   "dgrad_stream": "set_dgrad_stream", "autotune": "set_conv_autotune", "wgrad3": "set_wgrad3",
                   "splitk": "set_conv_splitk", "pipe_dgrad": "set_conv_pipe_dgrad", "wgrad_batch": "set_wgrad_batch",
                   "defer_direct": "set_defer_direct", "wgrad3_blocks": "set_wgrad3_blocks",
                   "conv3_stream": "set_conv3_stream", "head": "set_head1x1", "c8": "set_conv_c8", "c16": "set_conv_c16", "c3pro": "set_conv3_pro", "convT_stream": "set_convT_stream",
                   "halo_first": "set_halo_first", "halo_pipe": "set_halo_pipe", "wgrad_fast": "set_wgrad_fast", "wgrad_blocks": "set_wgrad_blocks"}
        for k, v in pins.items():
            if k in setters:
                getattr(_nat(), setters[k])(int(v))
        if pins.get("defer") == "0":
            from deeplearning_mpi_amd.ops.backend import NativeBackend

            NativeBackend.wgrad_defer = lambda self, on: None
    torch.manual_seed(0)
    shape = (cfg["cin"], cfg["image"], cfg["image"])
    if cfg["task"] == "cls":
        model = ARCHS[cfg["arch"]](num_classes=cfg["classes"]).to(dev)
        opt = SGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-5)
        crit = CrossEntropyLoss()
        x, y = device_batch("classification", cfg["batch"], dev, shape, cfg["classes"], seed=1234 + comm.rank)
        optname = "SGD(momentum=0.9, wd=1e-5)"
    else:
        model = UNet(out_classes=1, in_channels=cfg["cin"]).to(dev)
        opt = Adam(model.parameters(), lr=1e-4)
        crit = BCEWithLogitsLoss()
        x, y = device_batch("segmentation", cfg["batch"], dev, shape, seed=1234 + comm.rank)
        optname = "Adam(lr=1e-4) + clip_grad_norm(1.0)"
    model.precision = args.precision   # (read at the engine's first use, below)
    if args.rccl1:
        if world != 1:
            print("[bench] --rccl1 is a single-GPU option", file=sys.stderr, flush=True)
            sys.exit(2)
        from deeplearning_mpi_amd._ext import native
        from deeplearning_mpi_amd.parallel.comm import RcclCommunicator, rccl_channel_budget

        budget = rccl_channel_budget()
        nc = native().RcclComm(native().RcclComm.unique_id(), 0, 1, dev.index or 0)
        if args.rehearse > 0:
            class _Rehearsal(RcclCommunicator):
                def bucket_comm(self):
                    self.rbc = native().RehearsalBucketComm(self.c, args.rehearse_world, args.rehearse,
                                                            args.rehearse_lds, args.rehearse_gbps_ch,
                                                            args.rehearse_gbps_max, args.rehearse_lat_us)
                    return self.rbc

            rc = _Rehearsal(comm.info, dev, nc, budget=budget)
        else:
            rc = RcclCommunicator(comm.info, dev, nc, budget=budget)
        ddp = dl.DistributedDataParallel(model, bucket_cap_mb=args.bucket_mb, comm=rc, _force_reducer=True)
    else:
        ddp = dl.DistributedDataParallel(model, bucket_cap_mb=args.bucket_mb)

    def step():
        opt.zero_grad()
        out = ddp(x)
        if cfg["task"] == "cls":
            loss = crit(out, y)
            backward(loss)
        else:
            loss = crit(out.squeeze(1), y)
            backward(loss)
            clip_grad_norm_(model.parameters(), 1.0, optimizer=opt)
        opt.step()
        return loss

    if args.graph == "auto":
        from deeplearning_mpi_amd.apps.classification import use_graph

        args.graph = "1" if (not args.pyprof and not args.rehearse and not args.rccl1 and
                             use_graph(args, dev, pixels=cfg["batch"] * cfg["image"] * cfg["image"],
                                       comm_backend=getattr(comm, "backend", "single"))) else "0"
    args.graph = int(args.graph)
    if args.graph:
        from deeplearning_mpi_amd.utils.graphs import CapturedStep

        step = CapturedStep(step, warmup=2, inputs=(x, y))
        args.warmup = max(args.warmup, 3)   # 2 eager warmup calls + the capturing call stay untimed

    from deeplearning_mpi_amd._ext import native as _native

    red0 = _native().wgrad_reduce_launches()
    for i in range(args.warmup):
        step()
        if i == 0:   # one eager step: weight-gradient reduction launches (graph replays issue none)
            red_per_step = _native().wgrad_reduce_launches() - red0
    from deeplearning_mpi_amd.utils.profiler import ClockStamps

    clk = ClockStamps(dev)   # in-kernel shader clock over the timed steps (two 1024-wave stamp launches, paired per CU)
    comm.barrier()
    sync()
    t0 = time.perf_counter()
    clk.start()
    for _ in range(args.steps):
        loss = step()
    clk.stop()
    comm.barrier()
    sync()
    dt = time.perf_counter() - t0
    clock = clk.summary()
    myclk = torch.tensor([clock["sclk_mhz"] if clock else -1.0], dtype=torch.float64, device=dev)
    allclk = torch.empty(world, dtype=torch.float64, device=dev)
    comm.allgather(allclk, myclk)
    sclk_per_rank = [round(float(v), 1) if v > 0 else None for v in allclk.cpu()]
    # every rank's own wall time: the job's number is the slowest rank (MAX), min/max go to the JSON
    mine = torch.tensor([dt], dtype=torch.float64, device=dev)
    allt = torch.empty(world, dtype=torch.float64, device=dev)
    comm.allgather(allt, mine)
    per_rank_ms = [round(float(v) / args.steps * 1000, 3) for v in allt.cpu()]
    dt = float(allt.max().item())
    lossv = float(loss.item())
    global_batch = cfg["batch"] * world
    ips = global_batch * args.steps / dt
    # N > 1: a few untimed HIP-event-timed steps after the timed region answer "how much all-reduce
    # was left exposed after the backward pass" in the same JSON line
    if args.breakdown == 0 and (world > 1 or args.rehearse) and not args.graph:
        args.breakdown = 3
    bd_max = None
    if args.breakdown > 0 and not args.graph:
        # untimed extra steps: per-phase GPU time from HIP events (no host sync inside a step)
        from deeplearning_mpi_amd.utils.profiler import StepTimer

        tm = StepTimer()
        ddp.timer = tm
        for _ in range(args.breakdown):
            with tm.phase("step"):
                opt.zero_grad()
                with tm.phase("forward"):
                    out = ddp(x)
                    loss = crit(out, y) if cfg["task"] == "cls" else crit(out.squeeze(1), y)
                with tm.phase("backward"):   # includes comm_exposed
                    backward(loss)
                with tm.phase("optimizer"):
                    if cfg["task"] == "seg":
                        clip_grad_norm_(model.parameters(), 1.0, optimizer=opt)
                    opt.step()
        ddp.timer = None
        bd = {k: round(v, 3) for k, v in tm.summary().items()}
        bd.setdefault("comm_exposed", 0.0)
        bdt = torch.tensor([bd["comm_exposed"], bd["step"]], dtype=torch.float64, device=dev)
        comm.allreduce(bdt, "max")
        bd_max = {"comm_exposed": round(float(bdt[0]), 3), "step": round(float(bdt[1]), 3)}
        if comm.rank == 0:
            print(json.dumps({"breakdown_ms_per_step": bd, "max_over_ranks": bd_max,
                              "n_gpus": world, "config": args.config}), file=sys.stderr, flush=True)
    if args.pyprof > 0 and comm.rank == 0:
        import cProfile
        import io
        import pstats

        from deeplearning_mpi_amd.models import engine as _eng

        sync()
        pr, prb = cProfile.Profile(), cProfile.Profile()
        _eng.BWD_PROFILER = prb   # the engine backward runs on autograd's worker thread
        pr.enable()
        for _ in range(args.pyprof):
            step()
        pr.disable()
        _eng.BWD_PROFILER = None
        sync()
        for name, p_ in (("step (calling thread)", pr), ("engine backward (autograd thread)", prb)):
            buf = io.StringIO()
            pstats.Stats(p_, stream=buf).sort_stats("tottime").print_stats(40)
            print(f"[pyprof] {args.pyprof} steps, {name}, self time per function\n" + buf.getvalue(),
                  file=sys.stderr, flush=True)
    host_info = None
    if args.host_time > 0 and dev.type == "cuda":
        # host issue time of one step: the CPU time from calling step() to its return, each step
        # issued onto an idle GPU with empty queues (synchronised before and after, so a full launch
        # queue cannot block the host and inflate the number), vs the GPU time per step measured
        # above -- if the host needs less than the GPU, an eager pipelined step stays GPU-bound
        # 
        sync()
        issue = []
        t0 = time.perf_counter()
        for _ in range(args.host_time):
            a = time.perf_counter()
            step()
            issue.append(time.perf_counter() - a)
            sync()
        wall = time.perf_counter() - t0
        issue.sort()
        host_info = {"host_issue_ms_per_step_median": round(issue[len(issue) // 2] * 1e3, 3),
                     "host_issue_ms_per_step_max": round(issue[-1] * 1e3, 3),
                     "gpu_ms_per_step": round(dt / args.steps * 1e3, 3),
                     "wall_ms_per_step_during_probe_unpipelined": round(wall / args.host_time * 1e3, 3),
                     "host_over_gpu": round(issue[len(issue) // 2] / (dt / args.steps), 3)}
        if comm.rank == 0:
            print(json.dumps({"host_time": host_info, "config": args.config, "graph": bool(args.graph),
                              "rccl1": bool(args.rccl1)}), file=sys.stderr, flush=True)
    if args.mem and comm.rank == 0 and dev.type == "cuda":
        ms = torch.cuda.memory_stats(dev)
        print(json.dumps({"mem": {"peak_allocated_gb": round(ms.get("allocated_bytes.all.peak", 0) / 2 ** 30, 2),
                                  "peak_reserved_gb": round(ms.get("reserved_bytes.all.peak", 0) / 2 ** 30, 2),
                                  "alloc_retries": ms.get("num_alloc_retries", 0),
                                  "ooms": ms.get("num_ooms", 0),
                                  "device_total_gb": round(torch.cuda.get_device_properties(dev).total_memory / 2 ** 30, 1)}}),
              file=sys.stderr, flush=True)
    # one untimed step with every bucket all-reduce timed on the comm stream: when each bucket left,
    # how long it ran, its bus bandwidth, and how far the last one ended after the backward's compute
    bucket_info = None
    bc = getattr(ddp, "_bucket_comm", None)
    if args.bucket_probe and not args.graph and bc is not None and hasattr(bc, "set_timing"):
        bc.set_timing(True)
        step()
        sync()
        bc.set_timing(False)
        try:
            tm_ = bc.timings()
        except RuntimeError as e:   # an instrument: never fail the benchmark over it
            print(f"[bench] bucket probe failed: {e}", file=sys.stderr, flush=True)
            tm_ = {"buckets": []}
        bl = tm_["buckets"]
        # every rank takes part in both collectives below or in neither (a rank-local failure must not
        # leave the others waiting in an all-reduce)
        ok = torch.tensor([1.0 if (bl and "compute_end_ms" in tm_) else 0.0, float(len(bl))], device=dev)
        okmin = ok.clone()
        comm.allreduce(okmin, "min")
        okmax = ok.clone()
        comm.allreduce(okmax, "max")
        if okmin[0] > 0 and okmin[1] == okmax[1]:
            v = torch.tensor([b["dur_ms"] for b in bl] + [b["start_ms"] + b["dur_ms"] for b in bl] +
                             [tm_["compute_end_ms"]], dtype=torch.float64, device=dev)
            comm.allreduce(v, "max")   # every rank's slowest: the collective ends on the last rank
            nb = len(bl)
            durs, ends, cend = v[:nb].tolist(), v[nb:2 * nb].tolist(), float(v[-1])
            from deeplearning_mpi_amd.parallel.comm import bus_gbps

            bucket_info = {
                "buckets": [{"mb": round(b["bytes"] / 2 ** 20, 2), "start_ms": round(b["start_ms"], 3),
                             "dur_ms": round(d, 3),
                             "busbw_gbps": round(bus_gbps("allreduce", b["bytes"], d / 1e3, world), 1)}
                            for b, d in zip(bl, durs)],
                "backward_compute_end_ms": round(cend, 3),
                # > 0: all-reduce still running after the backward's compute (exposed); < 0: hidden
                "comm_tail_ms": round(max(ends) - cend, 3),
                "allreduce_ms_total": round(sum(durs), 3),
            }
    # distributed facts of this run: the world size RCCL itself reports, its CU (channel) budget,
    # the gradient bucket layout, per-rank step times and the exposed all-reduce (max over ranks)
    inner = getattr(ddp.comm, "inner", ddp.comm)
    native_comm = getattr(inner, "c", None)
    budget = getattr(inner, "budget", None) or {}
    cap = int(native_comm.max_ctas()) if native_comm is not None and hasattr(native_comm, "max_ctas") else 0
    dist_info = {
        "rccl_world_size": int(native_comm.size()) if native_comm is not None else None,
        "rccl_channels": (str(cap) if cap > 0 else os.environ.get("NCCL_MAX_NCHANNELS")) if native_comm is not None else None,
        "rccl_channel_calibration": budget.get("calibration"),
        "bucket_probe": bucket_info,
        "dgrad_stream_blocks": int(_native().dgs_blocks()),
        "wgrad_reduce_launches_per_step": int(red_per_step) if args.warmup > 0 else None,
        "bucket_mb": [round(b, 2) for b in ddp.bucket_sizes_mb()],
        "reducer": ddp.reducer is not None,
        "per_rank_ms_per_step": {"min": min(per_rank_ms), "max": max(per_rank_ms)},
        "comm_exposed_ms": bd_max["comm_exposed"] if bd_max else None,
        "sclk_mhz_per_rank": sclk_per_rank,
    }
    if host_info is not None:
        dist_info["host_time"] = host_info
    if args.rehearse > 0:
        rbc = ddp.comm.rbc
        dist_info["rehearsal"] = {
            "channels": args.rehearse, "world_modeled": args.rehearse_world, "lds_bytes": args.rehearse_lds,
            "gbps_per_channel": args.rehearse_gbps_ch, "gbps_max": args.rehearse_gbps_max,
            "latency_us": args.rehearse_lat_us,
            "modeled_allreduce_us_per_step": round(rbc.modeled_us_total() / max(1, rbc.buckets())
                                                   * len(ddp.bucket_sizes_mb()), 1),
            "buckets_launched": int(rbc.buckets()),
        }
    if comm.rank == 0:
        headline = args.config == "resnet50" and cfg == PRESETS["resnet50"]
        print(json.dumps({
            "metric": cfg["metric"],
            "value": round(ips, 2),
            "unit": "images/sec",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1000, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": (round(ips / BASELINE_VALUE, 4) if (BASELINE_VALUE and headline) else None),
            "dtype": "bf16" if model._be.act_dtype == torch.bfloat16 else str(model._be.act_dtype).replace("torch.", ""),
            "data": f"synthetic (random {'x'.join(map(str, shape))} inputs / "
                    f"{'labels' if cfg['task'] == 'cls' else 'binary masks'} generated on device, random-init weights)",
            "config": {"model": cfg["arch"], "global_batch": global_batch, "seq_len": None,
                       "image": cfg["image"], "in_channels": cfg["cin"], "per_gpu_batch": cfg["batch"],
                       "parallelism": f"dp{world}", "backend": comm.backend, "device": dev.type,
                       "optimizer": optname, "hipgraph": bool(args.graph),
                       "final_loss": round(lossv, 4)},
            "sclk_mhz": clock["sclk_mhz"] if clock else None,
            "clock": clock,
            "dist": dist_info,
        }), flush=True)
    dl.destroy_distributed()


if __name__ == "__main__":
    main()
