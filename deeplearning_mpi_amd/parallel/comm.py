"""Communicators: one object per process exposing the collectives the framework needs.

* :class:`RcclCommunicator` -- the GPU data plane: our native RCCL communicator (``_C.RcclComm``)
  over xGMI with its own comm stream; RCCL unique id distributed by MPI_Bcast (mpirun) or the
  launcher's TCPStore (torchrun).  No torch process group exists on this path.
* :class:`TorchCommunicator` -- ``torch.distributed`` gloo group (CPU tensors; tests, plumbing).
* :class:`MPICommunicator` -- host MPI collectives through ``_mpi`` (the CPU hello-world path).
* :class:`SingleCommunicator` -- world size 1, all collectives are no-ops.

``init_distributed()`` picks the launcher and backend; ``get_comm()`` returns the current one.
The reference uses ``dist.init_process_group('nccl'|'gloo')`` directly
(/root/reference/pytorch/hello_world/hello_world.py:33-39, resnet/main.py:147-153).
"""
from __future__ import annotations

import datetime
import os
import weakref

import torch
import torch.distributed as dist

from .bootstrap import LaunchInfo, detect_launcher, mpi_bring_up

_CURRENT = None


class Communicator:
    backend = "base"

    def __init__(self, info: LaunchInfo, device):
        self.info = info
        self.rank, self.world_size = info.rank, info.world_size
        self.local_rank = info.local_rank
        self.device = torch.device(device)

    # collectives on tensors (in place where applicable)
    def allreduce(self, t, op="sum"):
        raise NotImplementedError

    def broadcast(self, t, src=0):
        raise NotImplementedError

    def broadcast_async(self, t, src=0):
        """Start a broadcast; returns a callable that makes the caller's current stream wait for
        it (None when the broadcast already completed, as on host backends)."""
        self.broadcast(t, src)
        return None

    def allgather(self, out, t):
        raise NotImplementedError

    def reduce_scatter(self, out, t, op="sum"):
        raise NotImplementedError

    def alltoall(self, out, t):
        raise NotImplementedError

    def send(self, t, dst):
        raise NotImplementedError

    def recv(self, t, src):
        raise NotImplementedError

    def barrier(self):
        raise NotImplementedError

    def bucket_comm(self):
        """A ``_C.CommBase`` for the gradient reducer."""
        raise NotImplementedError

    def destroy(self):
        pass


class SingleCommunicator(Communicator):
    backend = "single"

    def allreduce(self, t, op="sum"):
        return t

    def broadcast(self, t, src=0):
        return t

    def allgather(self, out, t):
        out.view(-1).copy_(t.reshape(-1))
        return out

    def reduce_scatter(self, out, t, op="sum"):
        out.copy_(t.reshape(out.shape))
        return out

    def alltoall(self, out, t):
        out.copy_(t)
        return out

    def send(self, t, dst):
        raise RuntimeError("send with world_size 1")

    def recv(self, t, src):
        raise RuntimeError("recv with world_size 1")

    def barrier(self):
        pass


class RcclCommunicator(Communicator):
    backend = "rccl"

    def __init__(self, info, device, native_comm, control_group=None, budget=None):
        super().__init__(info, device)
        self.c = native_comm
        self.control = control_group
        # the CUs this communicator's channels take are withheld from the persistent streaming
        # data-gradient grid for as long as it exists (rccl_channel_budget)
        self.budget = budget if budget is not None else rccl_channel_budget()
        _LIVE_RCCL.add(self)
        _apply_dgs_budget()
        # a communicator dropped without destroy() releases its CUs when it is collected
        weakref.finalize(self, _apply_dgs_budget)

    def allreduce(self, t, op="sum"):
        self.c.allreduce(t, op, False)
        return t

    def broadcast(self, t, src=0):
        self.c.broadcast(t, src, False)
        return t

    def broadcast_async(self, t, src=0):
        # enqueued on the comm stream behind the compute stream's prior work; the returned fence
        # joins it back (no host block, capturable)
        self.c.broadcast(t, src, True)
        return self.c.wait

    def allgather(self, out, t):
        self.c.allgather(out, t.contiguous(), False)
        return out

    def reduce_scatter(self, out, t, op="sum"):
        self.c.reduce_scatter(out, t.contiguous(), op, False)
        return out

    def alltoall(self, out, t):
        self.c.alltoall(out, t.contiguous(), False)
        return out

    def send(self, t, dst):
        self.c.send(t, dst)

    def recv(self, t, src):
        self.c.recv(t, src)
        return t

    def barrier(self):
        self.c.barrier()

    def bucket_comm(self):
        from .._ext import native

        return native().RcclBucketComm(self.c)

    def destroy(self):
        self.c.destroy()
        self.control = None
        _LIVE_RCCL.discard(self)
        _apply_dgs_budget()


# RCCL communicators alive in this process (bench --rccl1 builds one beside init_distributed's).  The
# streaming data-gradient grid leaves room for the channels of every one of them: the smallest grid of
# the live budgets, the default (0) once none is left -- destroying one communicator must not hand the
# other's channels' CUs back to the persistent grid.  Weak: one dropped without destroy()
# leaves the set when it is collected, and its finalizer recomputes the grid.
_LIVE_RCCL = weakref.WeakSet()


def _apply_dgs_budget():
    from .._ext import native

    blocks = [int(c.budget["dgrad_stream_blocks"]) for c in _LIVE_RCCL]
    native().set_dgs_blocks(min(blocks) if blocks else 0)


def _make_torch_bucket_comm(group, world_size):
    from .._ext import native

    class _TorchBucketComm(native().CommBase):
        """Reducer backend over a torch.distributed group (gloo): async all-reduce per bucket,
        waited for (and averaged) at the end of the backward pass."""

        def __init__(self):
            super().__init__()
            self.works = []

        def allreduce_bucket(self, t, average):
            self.works.append((dist.all_reduce(t, group=group, async_op=True), t, average))

        def end_backward(self):
            for w, t, avg in self.works:
                w.wait()
                if avg:
                    t.div_(world_size)
            self.works.clear()

    return _TorchBucketComm()


class TorchCommunicator(Communicator):
    backend = "gloo"

    _OPS = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN,
            "prod": dist.ReduceOp.PRODUCT}

    def __init__(self, info, device, group=None):
        super().__init__(info, device)
        self.group = group

    def allreduce(self, t, op="sum"):
        if op == "avg":
            dist.all_reduce(t, dist.ReduceOp.SUM, group=self.group)
            t.div_(self.world_size)
        else:
            dist.all_reduce(t, self._OPS[op], group=self.group)
        return t

    def broadcast(self, t, src=0):
        dist.broadcast(t, src, group=self.group)
        return t

    def allgather(self, out, t):
        chunks = list(out.view(self.world_size, -1).unbind(0))
        dist.all_gather(chunks, t.reshape(-1).contiguous(), group=self.group)
        return out

    def reduce_scatter(self, out, t, op="sum"):
        full = t.reshape(self.world_size, -1).clone()
        self.allreduce(full, op)
        out.view(-1).copy_(full[self.rank])
        return out

    def alltoall(self, out, t):
        ins = list(t.reshape(self.world_size, -1).unbind(0))
        outs = list(out.view(self.world_size, -1).unbind(0))
        for r in range(self.world_size):   # gloo has no all_to_all: pairwise exchange
            if r == self.rank:
                outs[r].copy_(ins[r])
        reqs = []
        for r in range(self.world_size):
            if r != self.rank:
                reqs.append(dist.isend(ins[r].contiguous(), r, group=self.group))
                reqs.append(dist.irecv(outs[r], r, group=self.group))
        for q in reqs:
            q.wait()
        return out

    def send(self, t, dst):
        dist.send(t, dst, group=self.group)

    def recv(self, t, src):
        dist.recv(t, src, group=self.group)
        return t

    def barrier(self):
        dist.barrier(group=self.group)

    def bucket_comm(self):
        return _make_torch_bucket_comm(self.group, self.world_size)

    def destroy(self):
        if dist.is_initialized():
            dist.destroy_process_group()


class MPICommunicator(Communicator):
    """Host-side MPI collectives on CPU tensors (float32 / float64)."""

    backend = "mpi"

    def __init__(self, info, device="cpu"):
        super().__init__(info, device)
        from .._ext import mpi

        self.m = mpi()

    def allreduce(self, t, op="sum"):
        a = t.detach().cpu().contiguous()
        n = a.numpy()
        if a.dtype == torch.float64:
            self.m.allreduce_f64(n, "sum" if op == "avg" else op)
        else:
            n32 = n.astype("float32", copy=False)
            self.m.allreduce_f32(n32, "sum" if op == "avg" else op)
            a = torch.from_numpy(n32)
        if op == "avg":
            a /= self.world_size
        t.copy_(a)
        return t

    def broadcast(self, t, src=0):
        import numpy as np

        data = t.detach().cpu().contiguous().numpy().tobytes() if self.rank == src else b""
        buf = self.m.bcast_bytes(data, src)
        t.copy_(torch.from_numpy(np.frombuffer(buf, dtype=t.detach().cpu().numpy().dtype).copy()).view(t.shape))
        return t

    def send(self, t, dst):
        self.m.send_f32(t.detach().float().contiguous().numpy(), dst, 0)

    def recv(self, t, src):
        a = torch.empty(t.shape, dtype=torch.float32)
        self.m.recv_f32(a.numpy(), src, 0)
        t.copy_(a)
        return t

    def barrier(self):
        self.m.barrier()

    def destroy(self):
        self.m.finalize()


def _resolve_backend(backend: str) -> str:
    b = (backend or "auto").lower()
    if b == "auto":
        return "rccl" if torch.cuda.is_available() else "gloo"
    if b in ("nccl", "rccl"):
        return "rccl"
    if b in ("gloo", "mpi"):
        return b
    raise ValueError(f"unknown backend {backend!r}")


def init_distributed(backend: str = "auto", timeout_s: float = 1800.0, check: bool | None = None) -> Communicator:
    """Bring up ranks and the communicator. Safe to call once per process.

    check: wrap the communicator in the collective desync detector (parallel/debug.py); default
    from ``DLMPI_DESYNC_CHECK``.  timeout_s: control-plane timeout (a dead peer raises instead of
    hanging); the RCCL data plane has its own watchdog (``DLMPI_COMM_TIMEOUT``)."""
    global _CURRENT
    if _CURRENT is not None:
        return _CURRENT
    if check is None:
        check = os.environ.get("DLMPI_DESYNC_CHECK", "0") not in ("", "0")
    _CURRENT = _init(backend, timeout_s)
    if check and _CURRENT.world_size > 1:
        from .debug import CheckedCommunicator

        _CURRENT = CheckedCommunicator(_CURRENT)
    return _CURRENT


def _init(backend: str, timeout_s: float) -> Communicator:
    # cross-process GPU memory sharing on dmabuf-only hosts; must be set before the HSA runtime
    # starts (the first GPU call below)
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    info = detect_launcher()
    if info.launcher == "mpi":
        info = mpi_bring_up()
    be = _resolve_backend(backend)
    # gloo with GPU compute (gloo all-reduces CUDA tensors through host staging): rehearses the
    # multi-rank DDP path on a box with fewer GPUs than ranks, where RCCL refuses shared devices
    gloo_gpu = be == "gloo" and os.environ.get("DLMPI_GLOO_DEVICE", "cpu") == "cuda" and torch.cuda.is_available()
    if be == "rccl" or gloo_gpu:
        ndev = max(1, torch.cuda.device_count())   # does not initialise the GPU
        if info.local_rank < 0:
            info.local_rank = info.rank % ndev
        # one process per GPU; more local ranks than GPUs share devices round-robin (rehearsals)
        dev_idx = info.local_rank % ndev
        torch.cuda.set_device(dev_idx)
        device = torch.device("cuda", dev_idx)
    else:
        device = torch.device("cpu")
    if info.world_size == 1:
        return SingleCommunicator(info, device)
    if be == "mpi":
        return MPICommunicator(info, "cpu")
    if be == "gloo" or gloo_gpu:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=info.rank, world_size=info.world_size,
                                timeout=datetime.timedelta(seconds=timeout_s))
        return TorchCommunicator(info, device)
    # RCCL data plane: no torch process group at all, only the 128-byte unique id has to reach
    # every rank before ncclCommInitRank
    budget = rccl_channel_budget()
    from .._ext import native

    C = native()
    store = None
    if info.launcher == "mpi":
        # mpirun: the id travels by MPI_Bcast
        from .._ext import mpi

        uid = mpi().bcast_bytes(C.RcclComm.unique_id() if info.rank == 0 else b"", 0)
    else:
        uid, store = uid_via_store(info, C.RcclComm.unique_id, timeout_s)
    nc = C.RcclComm(uid, info.rank, info.world_size, device.index)
    if budget.get("mode") == "auto":
        # DLMPI_RCCL_CHANNELS=auto: the uncapped communicator only carries the calibration; the job's
        # communicator gets the chosen channel cap (calibrate_channels)
        cal = calibrate_channels(nc, info.rank, info.world_size, device)
        if cal["chosen"] > 0:
            fin = C.RcclComm(subcomm_uid(nc, info.rank, device), info.rank, info.world_size, device.index,
                             cal["chosen"])
            nc.destroy()
            nc = fin
        budget = dict(budget, dgrad_stream_blocks=int(os.environ.get("DLMPI_DGS_BLOCKS") or
                                                      max(64, 256 - (cal["chosen"] or 32))),
                      calibration=cal)
    return RcclCommunicator(info, device, nc, control_group=store, budget=budget)


def subcomm_uid(nc, rank, device) -> bytes:
    """A fresh RCCL unique id, made by rank 0 and broadcast over the live native communicator ``nc``
    (for a second communicator over the same ranks, e.g. with another channel cap)."""
    from .._ext import native

    C = native()
    raw = C.RcclComm.unique_id() if rank == 0 else bytes(128)
    t = torch.tensor(list(raw), dtype=torch.uint8, device=device)
    nc.broadcast(t, 0, False)
    return bytes(t.cpu().tolist())


def time_allreduce(nc, nbytes, device, iters=10, warmup=3, op="allreduce"):
    """Median time (s) of one ``op`` (allreduce / broadcast) of ``nbytes`` fp32 bytes on the native
    communicator ``nc``, bracketed by HIP events on the caller's stream (the collective's fences in and
    out), max over ranks."""
    t = torch.ones(max(1, nbytes // 4), dtype=torch.float32, device=device)
    fn = (lambda: nc.allreduce(t, "sum", False)) if op == "allreduce" else (lambda: nc.broadcast(t, 0, False))
    for _ in range(warmup):
        fn()
    times = []
    for _ in range(iters):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        times.append(a.elapsed_time(b) / 1e3)
    times.sort()
    med = torch.tensor([times[len(times) // 2]], dtype=torch.float64, device=device)
    nc.allreduce(med, "max", False)
    return float(med.item())


def bus_gbps(op, nbytes, seconds, world):
    """Bus bandwidth (GB/s, nccl-tests convention): all-reduce moves 2 (n-1)/n of the buffer per rank,
    broadcast the buffer once."""
    if seconds <= 0:
        return 0.0
    alg = nbytes / seconds / 1e9
    return alg * (2.0 * (world - 1) / world if op == "allreduce" else 1.0)


# candidate channel caps of DLMPI_RCCL_CHANNELS=auto, and the all-reduce size it calibrates at (the
# largest bucket cap, parallel/ddp.py)
AUTO_CAPS = (8, 16, 32)
AUTO_BYTES = 32 << 20
AUTO_FRACTION = 0.9


def calibrate_channels(nc, rank, world, device, caps=AUTO_CAPS, nbytes=AUTO_BYTES, iters=10) -> dict:
    """Measure all-reduce bus bandwidth of an ``nbytes`` buffer with each channel cap in ``caps`` (one
    temporary communicator each, ids broadcast over ``nc``) and with RCCL's own choice (``nc``), and
    pick the SMALLEST cap reaching AUTO_FRACTION of the best: each channel is a CU taken from the
    backward's compute while a bucket is in flight (profiles/r4_commload), so the fewest channels that
    carry the bucket at ~full bus bandwidth.  World size 1 has no bus: 0 (RCCL's choice) is kept."""
    from .._ext import native

    C = native()
    rows = [{"max_ctas": 0, "busbw_gbps": round(bus_gbps("allreduce", nbytes,
                                                           time_allreduce(nc, nbytes, device, iters), world), 1)}]
    for cap in caps:
        sub = C.RcclComm(subcomm_uid(nc, rank, device), rank, world, device.index, int(cap))
        rows.append({"max_ctas": int(cap),
                     "busbw_gbps": round(bus_gbps("allreduce", nbytes, time_allreduce(sub, nbytes, device, iters),
                                                  world), 1)})
        sub.destroy()
    return {"bytes": nbytes, "rows": rows, "chosen": choose_cap(rows, world)}


def choose_cap(rows, world, fraction=AUTO_FRACTION) -> int:
    """The smallest positive cap whose bus bandwidth is >= ``fraction`` of the best row's (0 = RCCL's
    own choice: world size 1, nothing measured, or no capped row good enough)."""
    best = max((r["busbw_gbps"] for r in rows), default=0.0)
    if world < 2 or best <= 0:
        return 0
    ok = [r["max_ctas"] for r in rows if r["max_ctas"] > 0 and r["busbw_gbps"] >= fraction * best]
    return min(ok) if ok else 0


# Measured by the one-GPU comm-load rehearsal (bench.py --rehearse, profiles/r4_commload): with a
# modeled 8-rank ring all-reduce after every gradient bucket, 8 channels cost the step 1.7 % (ResNet-50)
# / 2.1 % (ResNet-152) against the world-1 RCCL step -- the collective holds its CUs twice as long --
# while 16 and 32 channels cost 0.6 / 0.4 % and 1.1 / 0.3 %: within noise of each other, and 16 is the
# smallest budget at which the modeled collective is bus-bandwidth-, not channel-bound.
DEFAULT_RCCL_CHANNELS = 16


def rccl_channel_budget() -> dict:
    """How many CUs RCCL's kernels may take from the compute streams.

    Each RCCL channel is one workgroup (one CU) for the duration of a collective.  The gradient
    all-reduces run on the comm stream while the backward convolutions fill the other CUs, so the
    channel count is a CU budget: ``DLMPI_RCCL_CHANNELS`` (default 16 = 1/16 of the 256 CUs; 0 =
    leave RCCL its own choice) is exported as ``NCCL_MAX_NCHANNELS`` before the communicator is
    created (RCCL reads it at ``ncclCommInitRank``).  An explicit ``NCCL_MAX_NCHANNELS`` in the
    environment wins.  ``auto``: no process-wide cap; the communicator's own cap (maxCTAs) is the
    smallest of AUTO_CAPS that measures >= 90 % of the best all-reduce bus bandwidth at init
    (calibrate_channels).  The default (16) is the measured choice of the one-GPU comm-load rehearsal
    (``bench.py --rehearse``, profiles/r4_commload; see DEFAULT_RCCL_CHANNELS).

    The persistent streaming data-gradient kernel (conv1x1_dgrad_stream.hip) splits its work
    statically over one block per CU of 100-160 KB of LDS: a block that cannot start because an
    RCCL workgroup holds LDS on its CU would hold the whole kernel -- and the backward -- until the
    collective ends.  Its grid is therefore sized to the CUs the channels leave free
    (``dgrad_stream_blocks``; with RCCL's own, unknown, channel count: 256 - 32, RCCL's per-peer
    channel ceiling on this node size).  The communicator applies it natively for its lifetime
    (``RcclCommunicator``), so a later communicator with another budget takes effect.  Returns the
    effective settings (bench.py reports them)."""
    raw = os.environ.get("DLMPI_RCCL_CHANNELS", str(DEFAULT_RCCL_CHANNELS)).strip().lower()
    if raw == "auto" and "NCCL_MAX_NCHANNELS" not in os.environ:
        # per-communicator caps (ncclCommInitRankConfig maxCTAs) chosen by calibrate_channels at init
        return {"NCCL_MAX_NCHANNELS": None, "NCCL_MIN_NCHANNELS": os.environ.get("NCCL_MIN_NCHANNELS"),
                "dgrad_stream_blocks": int(os.environ.get("DLMPI_DGS_BLOCKS") or 256 - 32), "mode": "auto"}
    want = 0 if raw == "auto" else int(raw or 0)
    if want > 0 and "NCCL_MAX_NCHANNELS" not in os.environ:
        os.environ["NCCL_MAX_NCHANNELS"] = str(want)
    env = os.environ.get("NCCL_MAX_NCHANNELS")
    ch = int(env) if env else 32
    blocks = int(os.environ.get("DLMPI_DGS_BLOCKS") or max(64, 256 - ch))
    return {"NCCL_MAX_NCHANNELS": env, "NCCL_MIN_NCHANNELS": os.environ.get("NCCL_MIN_NCHANNELS"),
            "dgrad_stream_blocks": blocks}


_UID_ROUND = 0   # init_distributed -> destroy -> init_distributed in one process: a fresh key each time


def uid_via_store(info, make_uid, timeout_s=1800.0):
    """torchrun / env:// launch: the RCCL unique id goes through the launcher's c10d TCPStore (the
    elastic agent's store when torchrun shares it), obtained with the same env:// rendezvous
    ``init_process_group`` would use -- but no gloo/NCCL process group is created on top of it."""
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    store, _, _ = next(dist.rendezvous("env://", rank=info.rank, world_size=info.world_size,
                                       timeout=datetime.timedelta(seconds=timeout_s)))
    store.set_timeout(datetime.timedelta(seconds=timeout_s))
    global _UID_ROUND
    _UID_ROUND += 1
    key = f"dlmpi/rccl_uid/{os.environ.get('TORCHELASTIC_RESTART_COUNT', '0')}/{_UID_ROUND}"
    if info.rank == 0:
        uid = make_uid()
        store.set(key, uid)
    else:
        uid = store.get(key)
    return bytes(uid), store


def get_comm() -> Communicator:
    """Current communicator (a single-process one if init_distributed was never called)."""
    global _CURRENT
    if _CURRENT is None:
        info = detect_launcher()
        if info.world_size != 1:
            raise RuntimeError("multi-process launch detected: call init_distributed() first")
        dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
        _CURRENT = SingleCommunicator(info, dev)
    return _CURRENT


def destroy_distributed():
    global _CURRENT
    if _CURRENT is not None:
        _CURRENT.destroy()
    _CURRENT = None
