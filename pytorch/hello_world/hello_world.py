"""Communication hello-world (reference: pytorch/hello_world/hello_world.py:16-47).

Rank 0 sends a 1-element tensor to every other rank (the reference's P2P demo), and -- the
BASELINE.json config-1 plumbing check -- all ranks all-reduce their rank+1 and verify the sum.
Backends: nccl/rccl (GPU, our native RCCL communicator), gloo (CPU torch.distributed),
mpi (host MPI collectives through the native MPI module).  Launch with mpirun or torchrun:
    mpirun -n 2 python hello_world.py --backend gloo
    torchrun --nproc_per_node 2 hello_world.py --backend gloo
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))

import torch  # noqa: E402

from deeplearning_mpi_amd import parallel  # noqa: E402


def run(comm, op):
    rank, world = comm.rank, comm.world_size
    dev = comm.device
    ok = True
    if op in ("send", "both") and world > 1:
        tensor = torch.zeros(1, device=dev)
        if rank == 0:
            for rank_recv in range(1, world):
                comm.send(tensor, rank_recv)
                print("worker_{} sent data to Rank {}\n".format(0, rank_recv), flush=True)
        else:
            comm.recv(tensor, 0)
            print("worker_{} has received data from rank {}\n".format(rank, 0), flush=True)
    if op in ("allreduce", "both"):
        t = torch.full((4,), float(rank + 1), device=dev)
        comm.allreduce(t, "sum")
        want = world * (world + 1) / 2
        ok = bool(torch.allclose(t.cpu(), torch.full((4,), want)))
        print(f"rank {rank}/{world} [{comm.backend}] allreduce -> {t[0].item():g} (expected {want:g}): "
              f"{'OK' if ok else 'MISMATCH'}", flush=True)
    return ok


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--backend", type=str, default="nccl", choices=["nccl", "rccl", "gloo", "mpi"])
    ap.add_argument("--op", default="both", choices=["send", "allreduce", "both"])
    args = ap.parse_args()
    comm = parallel.init_distributed(args.backend)
    try:
        ok = run(comm, args.op)
    finally:
        parallel.destroy_distributed()
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
