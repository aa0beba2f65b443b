"""Collective desync / race detection (the reference has none: SURVEY.md §5.2, §5.3).

Distributed training hangs or silently corrupts when ranks issue DIFFERENT collectives -- the
reference's hazards are exactly that: a rank-local NaN ``continue`` that skips the backward's
all-reduce on one rank only (/root/reference/pytorch/unet/train.py:186-188) and a rank-0-only
evaluation on the DDP-wrapped model (K8, resnet/main.py:136-142).

:class:`CheckedCommunicator` wraps any communicator.  Before every collective each rank
fingerprints the call (sequence number, op, element count, dtype, root / reduction) and the ranks
compare fingerprints with one tiny all-reduce (max of (h, -h) == (h, -h) on every rank iff all
fingerprints agree).  On a mismatch every rank raises :class:`DesyncError` naming what each rank
was doing (gathered with one more small collective), instead of deadlocking inside RCCL or
reducing mismatched buffers.

Enable with ``init_distributed(..., check=True)`` or ``DLMPI_DESYNC_CHECK=1``.  The DDP wrapper
additionally verifies after every synchronised backward that all ranks launched the same number
of gradient buckets (a missed ``mark_ready`` on one rank).
"""
from __future__ import annotations

import hashlib

import torch

from .comm import Communicator



class DesyncError(RuntimeError):
    pass


def _h53(s: str) -> int:
    return int.from_bytes(hashlib.sha256(s.encode()).digest()[:6], "little")   # exact in float64


class CheckedCommunicator(Communicator):
    backend = "checked"

    def __init__(self, inner: Communicator):
        super().__init__(inner.info, inner.device)
        self.inner = inner
        self.backend = f"checked({inner.backend})"
        self.seq = 0
        self.history = []

    # ------------------------------------------------------------------ fingerprint exchange
    def _sig(self, name, t=None, **kw):
        parts = [f"#{self.seq}", name]
        if t is not None:
            parts += [f"numel={t.numel()}", f"dtype={str(t.dtype).replace('torch.', '')}"]
        parts += [f"{k}={v}" for k, v in sorted(kw.items())]
        return " ".join(parts)

    def _check(self, name, t=None, **kw):
        sig = self._sig(name, t, **kw)
        self.seq += 1
        self.history.append(sig)
        del self.history[:-64]
        h = float(_h53(sig))
        v = torch.tensor([h, -h], dtype=torch.float64, device=self._ctl_device())
        self.inner.allreduce(v, "max")
        if v[0].item() == h and v[1].item() == -h:
            return
        # gather every rank's signature for the error message
        code = torch.zeros(256, dtype=torch.float64, device=self._ctl_device())
        b = sig.encode()[:256]
        code[:len(b)] = torch.tensor(list(b), dtype=torch.float64)
        allc = torch.zeros(self.world_size * 256, dtype=torch.float64, device=self._ctl_device())
        self.inner.allgather(allc, code)
        lines = []
        for r in range(self.world_size):
            row = allc[r * 256:(r + 1) * 256].to(torch.int64).tolist()
            lines.append(f"  rank {r}: {bytes(c for c in row if c).decode(errors='replace')}")
        raise DesyncError("collective mismatch across ranks (would deadlock or corrupt):\n" + "\n".join(lines))

    def _ctl_device(self):
        return self.inner.device

    # ------------------------------------------------------------------ collectives
    def allreduce(self, t, op="sum"):
        self._check("allreduce", t, op=op)
        return self.inner.allreduce(t, op)

    def broadcast(self, t, src=0):
        self._check("broadcast", t, src=src)
        return self.inner.broadcast(t, src)

    def broadcast_async(self, t, src=0):
        self._check("broadcast", t, src=src)
        return self.inner.broadcast_async(t, src)

    def allgather(self, out, t):
        self._check("allgather", t)
        return self.inner.allgather(out, t)

    def reduce_scatter(self, out, t, op="sum"):
        self._check("reduce_scatter", t, op=op)
        return self.inner.reduce_scatter(out, t, op)

    def alltoall(self, out, t):
        self._check("alltoall", t)
        return self.inner.alltoall(out, t)

    def send(self, t, dst):   # point-to-point: only the pair participates, not checked collectively
        return self.inner.send(t, dst)

    def recv(self, t, src):
        return self.inner.recv(t, src)

    def barrier(self):
        self._check("barrier")
        return self.inner.barrier()

    def bucket_comm(self):
        return self.inner.bucket_comm()

    def destroy(self):
        self.inner.destroy()

    # ------------------------------------------------------------------ DDP step check
    def check_step(self, launched_buckets: int, step: int):
        """All ranks must have launched the same number of gradient buckets in this backward."""
        self._check("ddp_step", None, buckets=launched_buckets, step=step)
