"""The reference trainers on the GPU replay their steps from a captured hipGraph by default
(``--graph auto``); the replayed run must train bit-for-bit like the eager one,
including the eager ragged last batch."""
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args):
    env = dict(os.environ, PYTHONPATH=ROOT)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, *args], cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return r.stdout


@pytest.mark.parametrize("case", ["resnet", "unet"])
def test_app_graph_default_matches_eager(tmp_path, case):
    if case == "resnet":
        base = ["pytorch/resnet/main.py", "--synthetic", "--num_epochs", "1", "--batch_size", "32",
                "--synthetic_size", "176", "--workers", "0"]
        fname = "resnet_distributed.pth"
    else:
        base = ["pytorch/unet/train.py", "--synthetic", "--num_epochs", "1", "--batch_size", "4", "--image_size",
                "64", "--synthetic_size", "30", "--workers", "0", "--eval_every", "1", "--data_on_device", "0",
                "--log_dir", str(tmp_path / "logs")]
        fname = "model.pth"
    _run(base + ["--model_dir", str(tmp_path / "g")])                      # default: auto -> graph
    _run(base + ["--model_dir", str(tmp_path / "e"), "--graph", "0"])
    wg = torch.load(tmp_path / "g" / fname, weights_only=True)
    we = torch.load(tmp_path / "e" / fname, weights_only=True)
    for k in wg:
        assert torch.equal(wg[k], we[k]), k
