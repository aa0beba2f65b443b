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


class ClockStamps:
    """Mean shader clock of a GPU region, measured in-kernel: ``start()`` and
    ``stop()`` each launch a stamp kernel (util.hip clock_stamp_kernel: BLOCKS one-wave blocks writing
    {XCC id, HW_ID, s_memtime, s_memrealtime}) on the current stream; after a synchronisation
    ``summary()`` pairs a start and a stop stamp taken on the same CU (the shader-clock counters of
    different CUs are not synchronised): clock = d(memtime) / d(realtime) x 100 MHz per CU, the median
    over each XCD's CUs, then the mean over the XCDs and their min / max.  None where the native
    library is absent."""

    BLOCKS = 1024   # ~4 per CU, so that most CUs get a stamp at both ends

    def __init__(self, device):
        from .._ext import has_native, native

        self.C = native() if has_native() and torch.device(device).type == "cuda" else None
        if self.C is not None:
            self.buf = torch.zeros(2, self.BLOCKS, 4, dtype=torch.int64, device=device)

    def start(self):
        if self.C is not None:
            self.C.clock_stamp(self.buf[0])

    def stop(self):
        if self.C is not None:
            self.C.clock_stamp(self.buf[1])

    def summary(self):
        if self.C is None:
            return None
        return self.digest(self.buf.cpu().tolist())

    @staticmethod
    def digest(b):
        """b: [2][blocks][4] stamps (start, stop) -> the clock summary (pure, tested on the CPU)."""
        ends = [{}, {}]
        for k in (0, 1):
            for xcc, hw, mt, rt in b[k]:
                cu = (int(xcc), (int(hw) >> 8) & 0xFF)   # XCC + SE / SH / CU fields of HW_ID
                cur = ends[k].get(cu)
                # per CU: the earliest start stamp, the latest stop stamp
                if cur is None or (rt < cur[1] if k == 0 else rt > cur[1]):
                    ends[k][cu] = (mt, rt)
        per_xcd = {}
        for cu, (mt0, rt0) in ends[0].items():
            if cu in ends[1]:
                mt1, rt1 = ends[1][cu]
                if rt1 > rt0 and mt1 > mt0:
                    per_xcd.setdefault(cu[0], []).append((mt1 - mt0) / (rt1 - rt0) * 100.0)
        if not per_xcd:
            return None
        v = [sorted(c)[len(c) // 2] for c in per_xcd.values()]
        return {"sclk_mhz": round(sum(v) / len(v), 1), "sclk_mhz_min": round(min(v), 1),
                "sclk_mhz_max": round(max(v), 1), "xcds": len(v),
                "cus": sum(len(c) for c in per_xcd.values())}
