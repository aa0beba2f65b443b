"""Tracing / profiling helpers (the reference has none: SURVEY.md §5.1).

* :func:`range` -- roctx push/pop range (visible in ``rocprofv3 --marker-trace``), a no-op when
  libroctx64 is unavailable.
* :class:`StepTimer` -- HIP-event timing of named phases of a training step without host syncs
  inside the step; ``summary()`` synchronises once and returns per-phase milliseconds.
* :func:`throughput` -- images/sec helper used by the training apps and the benchmark.
"""
from __future__ import annotations

import contextlib
import ctypes
import time
from collections import defaultdict

import torch

_ROCTX = None


def _roctx():
    global _ROCTX
    if _ROCTX is None:
        _ROCTX = False
        for name in ("libroctx64.so", "/opt/rocm/lib/libroctx64.so"):
            try:
                lib = ctypes.CDLL(name)
                lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                lib.roctxRangePushA.restype = ctypes.c_int
                lib.roctxRangePop.restype = ctypes.c_int
                _ROCTX = lib
                break
            except OSError:
                continue
    return _ROCTX


@contextlib.contextmanager
def range(name: str):  # noqa: A001 - mirrors torch.cuda.nvtx.range
    lib = _roctx()
    if lib:
        lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        if lib:
            lib.roctxRangePop()


class StepTimer:
    """Accumulate GPU time per named phase with HIP events (no synchronisation while timing)."""

    def __init__(self, enabled: bool = True):
        self.enabled = enabled and torch.cuda.is_available()
        self._ev = defaultdict(list)
        self._wall = defaultdict(float)

    @contextlib.contextmanager
    def phase(self, name: str):
        if not self.enabled:
            t0 = time.perf_counter()
            with range(name):
                yield
            self._wall[name] += time.perf_counter() - t0
            return
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        s.record()
        with range(name):
            yield
        e.record()
        self._ev[name].append((s, e))

    def summary(self) -> dict:
        out = {}
        if self.enabled:
            torch.cuda.synchronize()
            for k, v in self._ev.items():
                out[k] = sum(s.elapsed_time(e) for s, e in v) / max(1, len(v))
        for k, v in self._wall.items():
            out[k] = v * 1e3
        return out

    def reset(self):
        self._ev.clear()
        self._wall.clear()


def throughput(images: int, seconds: float) -> float:
    return images / max(seconds, 1e-12)
