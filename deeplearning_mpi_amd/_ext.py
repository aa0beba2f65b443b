"""Loader for the in-tree native extensions.

``native()`` returns the ``_C`` module (gfx950 kernels, RCCL comm, reducer).  On a machine with a
GPU the extension is REQUIRED: if it is missing or fails to load we raise instead of silently
falling back to eager PyTorch, so a GPU run can never pass on a non-native path.  On a CPU-only
host the framework runs its torch reference backend (used by the CPU test-suite) and ``native()``
raises only when something actually asks for GPU kernels.
"""
from __future__ import annotations

import importlib
import os

_C = None
_ERR = None
_MPI = None
_MPI_ERR = None


def _load():
    global _C, _ERR
    if _C is not None or _ERR is not None:
        return
    try:
        import torch  # noqa: F401  (loads libtorch / libc10_hip / librccl first)

        _C = importlib.import_module("deeplearning_mpi_amd._C")
    except Exception as e:  # pragma: no cover - depends on the build state
        _ERR = e
        if os.environ.get("DLMPI_AUTOBUILD", "1") == "1":
            try:
                from . import build

                build.build()
                _C = importlib.import_module("deeplearning_mpi_amd._C")
                _ERR = None
            except Exception as e2:
                _ERR = e2


def native():
    """The native module; raises a RuntimeError naming the cause if it is unavailable."""
    _load()
    if _C is None:
        raise RuntimeError(
            "deeplearning_mpi_amd native extension (_C) is not available: "
            f"{_ERR!r}. Build it with `python -m deeplearning_mpi_amd.build`.")
    return _C


def has_native() -> bool:
    _load()
    return _C is not None


def mpi():
    """The MPI bootstrap module (``_mpi``), or raise."""
    global _MPI, _MPI_ERR
    if _MPI is None and _MPI_ERR is None:
        try:
            _MPI = importlib.import_module("deeplearning_mpi_amd._mpi")
        except Exception as e:  # pragma: no cover
            _MPI_ERR = e
    if _MPI is None:
        raise RuntimeError(f"MPI bootstrap module unavailable: {_MPI_ERR!r}")
    return _MPI


def gpu_required() -> bool:
    """True when a GPU is visible: then the native path is mandatory."""
    import torch

    return torch.cuda.is_available()
