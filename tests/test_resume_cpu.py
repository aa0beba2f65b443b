"""Exact resume: 2 epochs, then ``--resume`` for the 3rd, must end bit-for-bit
where 3 uninterrupted epochs end -- weights, BatchNorm buffers and optimizer state -- for both
reference trainers, launched as 2 gloo ranks with torchrun.  The main checkpoint file keeps the
reference layout (``module.``-prefixed state_dict); the resume state lives in the sidecar."""
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
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nproc_per_node", "2", "--master_addr",
                        "127.0.0.1", "--master_port", str(_port()), script, "--synthetic", "--device", "cpu",
                        "--backend", "gloo", "--workers", "0", "--eval_every", "1", *args],
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


CASES = {
    "resnet": ("pytorch/resnet/main.py", "resnet_distributed.pth",
               ["--batch_size", "4", "--synthetic_size", "16"]),
    "unet": ("pytorch/unet/train.py", "model.pth",
             ["--batch_size", "2", "--image_size", "32", "--synthetic_size", "10"]),
}


@pytest.mark.parametrize("case", sorted(CASES))
def test_two_epochs_plus_resume_equals_three_epochs(tmp_path, case):
    script, fname, extra = CASES[case]
    if case == "unet":
        extra = extra + ["--log_dir", str(tmp_path / "logs")]
    a, b = tmp_path / "a", tmp_path / "b"
    _run(script, ["--num_epochs", "3", "--model_dir", str(a), *extra])
    _run(script, ["--num_epochs", "2", "--model_dir", str(b), *extra])
    out = _run(script, ["--num_epochs", "3", "--model_dir", str(b), "--resume", *extra])
    if case == "resnet":
        assert "Epoch 2 completed" in out and "Epoch 0 completed" not in out   # continued, not restarted
    wa = torch.load(a / fname, weights_only=True)
    wb = torch.load(b / fname, weights_only=True)
    assert wa.keys() == wb.keys() and all(k.startswith("module.") for k in wa)
    for k in wa:
        assert torch.equal(wa[k], wb[k]), k
    sa = torch.load(str(a / fname) + ".state", weights_only=True)
    sb = torch.load(str(b / fname) + ".state", weights_only=True)
    assert sa["next_epoch"] == sb["next_epoch"] == 3
    oa, ob = _flat_state(sa["optimizer"]["state"]), _flat_state(sb["optimizer"]["state"])
    assert oa and oa.keys() == ob.keys()
    for k in oa:
        assert torch.equal(oa[k], ob[k]), k
