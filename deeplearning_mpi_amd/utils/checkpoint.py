"""Checkpoints, layout-compatible with the reference.

The main file is exactly what the reference writes -- ``torch.save(ddp_model.state_dict(), path)``
(/root/reference/pytorch/resnet/main.py:139, unet/train.py:216): a flat dict of fp32 tensors whose
keys carry the ``module.`` prefix -- so reference checkpoints load here and ours load there.
Resume state (optimizer, next epoch, sampler epoch, RNG states: :func:`resume_state`) goes to a
sidecar ``<path>.state`` so the main file layout never changes; the apps write it with every
checkpoint and ``--resume`` continues from it exactly (tests/test_resume_cpu.py).  Only GLOBAL rank 0 writes (the reference gates on
LOCAL_RANK, which collides across nodes on a shared filesystem).
Loading uses ``torch.load(..., weights_only=True)`` and accepts either key style.

Crash consistency: the sidecar records the SHA-256 of the weights file it belongs to.  A save keeps
the previous sidecar as ``<path>.state.prev`` when it belongs to the weights still on disk (after an
interrupted save it may not: then the existing ``.state.prev`` is kept), then puts the new sidecar
and finally the new weights in place.  A crash anywhere in between leaves weights
whose own sidecar is on disk under one of the two names, and ``load_checkpoint`` takes the one whose
hash matches -- never new weights with an old optimizer state / epoch, and never an already trained
checkpoint restarted from epoch 0.
"""
from __future__ import annotations

import hashlib
import os
import random
import warnings

import numpy as np
import torch


def _sha256(path) -> str:
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for chunk in iter(lambda: f.read(1 << 22), b""):
            h.update(chunk)
    return h.hexdigest()


def _sidecar_matches(state_path, weights_path) -> bool:
    """True if the sidecar belongs to the weights file on disk (or there are no weights, or the
    sidecar predates the hash)."""
    if not os.path.exists(weights_path):
        return True
    try:
        want = torch.load(state_path, map_location="cpu", weights_only=True).get("weights_sha256")
    except Exception:   # unreadable (torn) sidecar: never rotate it over a good one
        return False
    return want is None or want == _sha256(weights_path)


def save_checkpoint(model, path, optimizer=None, extra=None, rank=None):
    if rank is None:
        from ..parallel.comm import get_comm

        rank = get_comm().rank
    if rank != 0:
        return None
    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)
    sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    tmp = path + ".tmp"
    torch.save(sd, tmp)
    if optimizer is not None or extra:
        state = dict(extra or {})
        if optimizer is not None:
            state["optimizer"] = optimizer.state_dict()
        state["weights_sha256"] = _sha256(tmp)
        torch.save(state, path + ".state.tmp")
        # keep the resume state of the weights still on disk as .state.prev -- but only if .state IS
        # theirs: after an interrupted save .state may belong to weights that never landed, and then
        # the existing .state.prev is the one to keep
        if os.path.exists(path + ".state") and _sidecar_matches(path + ".state", path):
            os.replace(path + ".state", path + ".state.prev")
        os.replace(path + ".state.tmp", path + ".state")   # sidecar before weights (module docstring)
    os.replace(tmp, path)
    return path


def _adapt_keys(sd, want_prefix):
    has = all(k.startswith("module.") for k in sd)
    if want_prefix and not has:
        return {"module." + k: v for k, v in sd.items()}
    if not want_prefix and has:
        return {k[len("module."):]: v for k, v in sd.items()}
    return sd


def load_checkpoint(model, path, map_location=None, optimizer=None, strict=True):
    """Load weights (and, when present, the sidecar resume state). Returns the sidecar dict."""
    if map_location is None:
        p = next(model.parameters())
        map_location = p.device
    sd = torch.load(path, map_location=map_location, weights_only=True)
    want_prefix = all(k.startswith("module.") for k in model.state_dict())
    sd = _adapt_keys(sd, want_prefix)
    with torch.no_grad():
        model.load_state_dict(sd, strict=strict)
    meta = {}
    cands = [c for c in (path + ".state", path + ".state.prev") if os.path.exists(c)]
    if cands:
        digest = _sha256(path)
        for c in cands:
            m = torch.load(c, map_location=map_location, weights_only=True)
            want = m.get("weights_sha256")
            if want is None or want == digest:
                meta = m
                break
        else:
            warnings.warn(f"no resume state of {path} matches its weights (interrupted save?): "
                          "starting from epoch 0 with fresh optimizer state")
        if optimizer is not None and "optimizer" in meta:
            optimizer.load_state_dict(meta["optimizer"])
    from .arena import arena_of

    a = arena_of(next(iter(model.parameters())))
    if a is not None:
        a.mark_updated()
    return meta


def rng_state() -> dict:
    """Host (torch / numpy / python) and device RNG states, as tensors and plain numbers only so
    the sidecar loads with ``weights_only=True``."""
    np_s = np.random.get_state()
    py = random.getstate()
    st = {"torch": torch.get_rng_state(),
          "numpy": {"keys": torch.from_numpy(np.asarray(np_s[1], dtype=np.int64)), "pos": int(np_s[2]),
                    "has_gauss": int(np_s[3]), "gauss": float(np_s[4])},
          "python": {"version": int(py[0]), "state": torch.tensor(py[1], dtype=torch.int64), "gauss": py[2]}}
    if torch.cuda.is_available() and torch.cuda.is_initialized():
        st["cuda"] = [t.cpu() for t in torch.cuda.get_rng_state_all()]
    return st


def set_rng_state(st: dict):
    if not st:
        return
    torch.set_rng_state(st["torch"].cpu())
    n = st["numpy"]
    np.random.set_state(("MT19937", n["keys"].cpu().numpy().astype(np.uint32), n["pos"], n["has_gauss"], n["gauss"]))
    p = st["python"]
    random.setstate((p["version"], tuple(int(v) for v in p["state"].tolist()), p["gauss"]))
    if "cuda" in st and torch.cuda.is_available():
        torch.cuda.set_rng_state_all([t.cpu() for t in st["cuda"]])


def resume_state(next_epoch: int, **more) -> dict:
    """Sidecar payload: the epoch to continue with, the sampler epoch and the RNG states."""
    return dict(next_epoch=int(next_epoch), sampler_epoch=int(next_epoch), rng=rng_state(), **more)
