"""Rank bootstrap: mpirun (MPICH Hydra / Open MPI), torchrun, or a single process.

Replaces the reference's "read LOCAL_RANK/RANK/WORLD_SIZE at import and raise"
(/root/reference/pytorch/resnet/main.py:17-23, unet/train.py:20-25) and its torchrun-only launch
(unet/run.sh:100-112).  Under ``mpirun`` the ranks come from MPI itself and the control-plane
rendezvous address is broadcast with MPI_Bcast, so no MASTER_ADDR/PORT has to be configured.
Detection order: MPI environment -> torchrun environment -> single process.
"""
from __future__ import annotations

import os
import socket
from dataclasses import dataclass


@dataclass
class LaunchInfo:
    launcher: str          # "mpi" | "torchrun" | "single"
    rank: int
    world_size: int
    local_rank: int
    local_world_size: int


def _env_int(*names, default=None):
    for n in names:
        v = os.environ.get(n)
        if v is not None and v != "":
            return int(v)
    return default


def detect_launcher() -> LaunchInfo:
    """Rank info from the environment only (no MPI call, no GPU touch)."""
    mrank = _env_int("OMPI_COMM_WORLD_RANK", "PMI_RANK", "PMIX_RANK", "MV2_COMM_WORLD_RANK")
    if mrank is not None:
        msize = _env_int("OMPI_COMM_WORLD_SIZE", "PMI_SIZE", "MV2_COMM_WORLD_SIZE", default=1)
        lrank = _env_int("OMPI_COMM_WORLD_LOCAL_RANK", "MPI_LOCALRANKID", "MV2_COMM_WORLD_LOCAL_RANK", default=-1)
        lsize = _env_int("OMPI_COMM_WORLD_LOCAL_SIZE", "MPI_LOCALNRANKS", "MV2_COMM_WORLD_LOCAL_SIZE", default=-1)
        return LaunchInfo("mpi", mrank, msize, lrank, lsize)
    if "RANK" in os.environ and "WORLD_SIZE" in os.environ:
        return LaunchInfo("torchrun", int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"]),
                          _env_int("LOCAL_RANK", default=0), _env_int("LOCAL_WORLD_SIZE", default=1))
    return LaunchInfo("single", 0, 1, 0, 1)


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("", 0))
        return s.getsockname()[1]


def _my_addr() -> str:
    addr = os.environ.get("DLMPI_MASTER_ADDR")
    if addr:
        return addr
    try:
        a = socket.gethostbyname(socket.gethostname())
        if a and not a.startswith("127."):
            return a
    except OSError:
        pass
    return "127.0.0.1"


def mpi_bring_up() -> LaunchInfo:
    """MPI_Init, rank/size/local rank from MPI, and the control-plane rendezvous exported as the
    torchrun-style environment (RANK, WORLD_SIZE, LOCAL_RANK, MASTER_ADDR, MASTER_PORT)."""
    from .._ext import mpi

    m = mpi()
    rank, size = m.init()
    lrank, lsize = m.local_rank()
    if rank == 0:
        addr = os.environ.get("MASTER_ADDR") or _my_addr()
        port = os.environ.get("MASTER_PORT") or str(_free_port())
        payload = f"{addr}:{port}".encode()
    else:
        payload = b""
    addr, port = m.bcast_bytes(payload, 0).decode().split(":")
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(size), "LOCAL_RANK": str(lrank),
                       "LOCAL_WORLD_SIZE": str(lsize), "MASTER_ADDR": addr, "MASTER_PORT": port})
    return LaunchInfo("mpi", rank, size, lrank, lsize)
