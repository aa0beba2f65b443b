"""Exact resume: 2 epochs, then ``--resume`` for the 3rd, must end
bit-for-bit where 3 uninterrupted epochs end -- weights, BatchNorm buffers and optimizer state -- for
both reference trainers, launched as 2 gloo ranks with torchrun.  The main checkpoint file keeps the
reference layout (``module.``-prefixed state_dict); the resume state lives in the sidecar.

The ``*_cifar_host`` cases run the host CIFAR-10 pipeline (a small CIFAR binary written here,
RandomCrop + flip augmentation, 2 DataLoader workers per rank, rank-0-only evaluation) -- the path on
which the per-rank augmentation generator and rank 0's evaluation draws used to break exactness.
Both reference variants run: main.py (evaluate after the epoch) and resnet.py (evaluate before)."""
import os
import socket
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(script, args):
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    base = ["--device", "cpu", "--backend", "gloo", "--eval_every", "1"]
    if "--data_root" not in args:
        base += ["--synthetic", "--workers", "0"]
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nproc_per_node", "2", "--master_addr",
                        "127.0.0.1", "--master_port", str(_port()), script, *base, *args],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return r.stdout


def _flat_state(d):
    out = {}
    for k, v in d.items():
        if isinstance(v, dict):
            out.update({f"{k}.{kk}": vv for kk, vv in _flat_state(v).items()})
        elif isinstance(v, torch.Tensor):
            out[k] = v
    return out


def _fake_cifar(root, n=12):
    """A CIFAR-10 binary release with ``n`` random images per file (same format as the real one)."""
    import numpy as np

    d = root / "cifar-10-batches-bin"
    d.mkdir(parents=True, exist_ok=True)
    rng = np.random.default_rng(7)
    for f in [f"data_batch_{i}.bin" for i in range(1, 6)] + ["test_batch.bin"]:
        rows = np.concatenate([rng.integers(0, 10, (n, 1)), rng.integers(0, 256, (n, 3072))], 1).astype(np.uint8)
        rows.tofile(d / f)
    return root


CASES = {
    "resnet": ("pytorch/resnet/main.py", "resnet_distributed.pth",
               ["--batch_size", "4", "--synthetic_size", "16"]),
    "resnet_cifar_host": ("pytorch/resnet/main.py", "resnet_distributed.pth",
                          ["--batch_size", "6", "--workers", "2", "--data_on_device", "0"]),
    "resnet_variant_b_cifar_host": ("pytorch/resnet/resnet.py", "resnet_distributed.pth",
                                    ["--batch_size", "6", "--workers", "2", "--data_on_device", "0",
                                     "--test_batch_size", "8"]),
    "unet": ("pytorch/unet/train.py", "model.pth",
             ["--batch_size", "2", "--image_size", "32", "--synthetic_size", "10"]),
}


@pytest.mark.parametrize("case", sorted(CASES))
def test_two_epochs_plus_resume_equals_three_epochs(tmp_path, case):
    script, fname, extra = CASES[case]
    if case == "unet":
        extra = extra + ["--log_dir", str(tmp_path / "logs")]
    if "cifar_host" in case:
        extra = extra + ["--data_root", str(_fake_cifar(tmp_path / "data"))]
    a, b = tmp_path / "a", tmp_path / "b"
    _run(script, ["--num_epochs", "3", "--model_dir", str(a), *extra])
    _run(script, ["--num_epochs", "2", "--model_dir", str(b), *extra])
    out = _run(script, ["--num_epochs", "3", "--model_dir", str(b), "--resume", *extra])
    if case.startswith("resnet"):
        assert "Epoch 2 completed" in out and "Epoch 0 completed" not in out   # continued, not restarted
    wa = torch.load(a / fname, weights_only=True)
    wb = torch.load(b / fname, weights_only=True)
    assert wa.keys() == wb.keys() and all(k.startswith("module.") for k in wa)
    for k in wa:
        assert torch.equal(wa[k], wb[k]), k
    sa = torch.load(str(a / fname) + ".state", weights_only=True)
    sb = torch.load(str(b / fname) + ".state", weights_only=True)
    # resnet.py evaluates + saves BEFORE training an epoch: its last checkpoint of a 3-epoch run is the
    # one written at the start of epoch 2 (the resumed run re-trained epoch 1 from the epoch-1 save)
    assert sa["next_epoch"] == sb["next_epoch"] == (2 if "variant_b" in case else 3)
    oa, ob = _flat_state(sa["optimizer"]["state"]), _flat_state(sb["optimizer"]["state"])
    assert oa and oa.keys() == ob.keys()
    for k in oa:
        assert torch.equal(oa[k], ob[k]), k


def test_checkpoint_sidecar_survives_interrupted_save(tmp_path):
    """a crash between the sidecar and the weights rename must leave a loadable resume
    state for the weights still on disk (the previous sidecar, kept as <path>.state.prev), and the
    finished save must load its own."""
    import os

    import torch

    from deeplearning_mpi_amd.utils.checkpoint import load_checkpoint, save_checkpoint

    m = torch.nn.Linear(4, 3)
    p = str(tmp_path / "ck.pth")
    save_checkpoint(m, p, extra={"next_epoch": 1}, rank=0)
    with torch.no_grad():
        m.weight.add_(1.0)
    # an interrupted second save: sidecar of epoch 2 in place, weights of epoch 1 still on disk
    orig = os.replace

    def crash_on_weights(src, dst):
        if dst == p:
            raise KeyboardInterrupt("simulated crash")
        return orig(src, dst)

    os.replace = crash_on_weights
    try:
        save_checkpoint(m, p, extra={"next_epoch": 2}, rank=0)
    except KeyboardInterrupt:
        pass
    finally:
        os.replace = orig
    m2 = torch.nn.Linear(4, 3)
    meta = load_checkpoint(m2, p, map_location="cpu")
    assert meta.get("next_epoch") == 1   # the weights on disk are epoch 1's, and so is the state
    save_checkpoint(m, p, extra={"next_epoch": 2}, rank=0)
    assert load_checkpoint(m2, p, map_location="cpu").get("next_epoch") == 2
    assert torch.equal(m2.weight, m.weight)


def test_checkpoint_sidecar_survives_two_interrupted_saves(tmp_path):
    """two saves interrupted in the same window (after the sidecar, before the weights)
    must not rotate the first interrupted save's stale sidecar over the only one matching the weights
    on disk: the load still resumes epoch 1's state, not epoch 0 with a fresh optimizer."""
    import os

    import torch

    from deeplearning_mpi_amd.utils.checkpoint import load_checkpoint, save_checkpoint

    m = torch.nn.Linear(4, 3)
    p = str(tmp_path / "ck.pth")
    save_checkpoint(m, p, extra={"next_epoch": 1}, rank=0)
    orig = os.replace

    def crash_on_weights(src, dst):
        if dst == p:
            raise KeyboardInterrupt("simulated crash")
        return orig(src, dst)

    for ep in (2, 3):
        with torch.no_grad():
            m.weight.add_(1.0)
        os.replace = crash_on_weights
        try:
            save_checkpoint(m, p, extra={"next_epoch": ep}, rank=0)
        except KeyboardInterrupt:
            pass
        finally:
            os.replace = orig
    m2 = torch.nn.Linear(4, 3)
    with __import__("warnings").catch_warnings():
        __import__("warnings").simplefilter("error")   # "no resume state matches" would be a failure
        meta = load_checkpoint(m2, p, map_location="cpu")
    assert meta.get("next_epoch") == 1
    save_checkpoint(m, p, extra={"next_epoch": 4}, rank=0)
    assert load_checkpoint(m2, p, map_location="cpu").get("next_epoch") == 4
    assert torch.equal(m2.weight, m.weight)
