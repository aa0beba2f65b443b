"""The reference entry points (same paths, flags and artefacts) run end to end on CPU / gloo:
pytorch/resnet/main.py and resnet.py (1 epoch of synthetic data, evaluation, module.-prefixed
checkpoint), pytorch/unet/train.py (log file format of train.py:44-57, Dice eval, checkpoint),
the --benchmark_steps / --precision flags, and a 2-rank torchrun launch in which only global
rank 0 writes the checkpoint (SURVEY.md §5.2 hazard b)."""
import glob
import os
import socket
import subprocess
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, timeout=600, env_extra=None):
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update(env_extra or {})
    r = subprocess.run(args, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return r.stdout


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


COMMON = ["--synthetic", "--device", "cpu", "--backend", "gloo", "--workers", "0"]


def test_resnet_main_one_epoch_and_checkpoint(tmp_path):
    out = _run([sys.executable, "pytorch/resnet/main.py", *COMMON, "--num_epochs", "1", "--batch_size", "8",
                "--synthetic_size", "32", "--model_dir", str(tmp_path)])
    assert "Epoch: 0, Accuracy:" in out and "Epoch 0 completed" in out
    sd = torch.load(tmp_path / "resnet_distributed.pth", weights_only=True)
    assert len(sd) == 122 and all(k.startswith("module.") for k in sd)


def test_resnet_variant_b_resume(tmp_path):
    _run([sys.executable, "pytorch/resnet/resnet.py", *COMMON, "--num_epochs", "1", "--batch_size", "8",
          "--synthetic_size", "16", "--model_dir", str(tmp_path)])
    out = _run([sys.executable, "pytorch/resnet/resnet.py", *COMMON, "--num_epochs", "1", "--batch_size", "8",
                "--synthetic_size", "16", "--model_dir", str(tmp_path), "--resume"])
    assert "Accuracy" in out


def test_benchmark_steps_and_fp32_precision():
    out = _run([sys.executable, "pytorch/resnet/main.py", *COMMON, "--benchmark_steps", "2", "--batch_size", "4",
                "--precision", "fp32"])
    assert "images/sec" in out


def test_unet_train_log_format_and_checkpoint(tmp_path):
    logs = tmp_path / "logs"
    out = _run([sys.executable, "pytorch/unet/train.py", *COMMON, "--num_epochs", "2", "--batch_size", "2",
                "--image_size", "32", "--synthetic_size", "10", "--eval_every", "1", "--log_dir", str(logs),
                "--model_dir", str(tmp_path)])
    assert "Dice Score" in out and "TRAINING COMPLETED" in out
    (log,) = glob.glob(str(logs / "training_log_*.log"))
    txt = open(log).read()
    for needle in ("Batch size: 2", "Learning rate: 0.0001", "Number of epochs: 2", "World size: 1",
                   "Started training at", "Epoch 1 | Loss:", "| Duration:", "Epoch 2 | Dice Score:"):
        assert needle in txt, needle
    sd = torch.load(tmp_path / "model.pth", weights_only=True)
    assert len(sd) == 136 and all(k.startswith("module.") for k in sd)


def test_torchrun_two_ranks_rank0_writes_checkpoint(tmp_path):
    out = _run([sys.executable, "-m", "torch.distributed.run", "--nproc_per_node", "2", "--master_addr", "127.0.0.1",
                "--master_port", str(_port()), "pytorch/resnet/main.py", *COMMON, "--num_epochs", "1",
                "--batch_size", "4", "--synthetic_size", "16", "--model_dir", str(tmp_path)])
    assert out.count("Epoch 0 completed") == 2
    assert os.listdir(tmp_path) == ["resnet_distributed.pth"] or sorted(os.listdir(tmp_path)) == sorted(
        ["resnet_distributed.pth", "resnet_distributed.pth.state"])


def _fake_cifar_bin(root, per_file=6):
    import numpy as np

    d = root / "cifar-10-batches-bin"
    d.mkdir(parents=True)
    g = np.random.default_rng(0)
    for name in [f"data_batch_{i}.bin" for i in range(1, 6)] + ["test_batch.bin"]:
        rec = g.integers(0, 256, size=(per_file, 3073), dtype=np.uint8)
        rec[:, 0] %= 10
        rec.tofile(d / name)


def test_resnet_cifar_device_resident_and_dataloader_paths(tmp_path):
    """Real-data path on a small CIFAR-10 binary-format file set: the device-resident pipeline
    (--data_on_device 1; on CPU it runs the torch reference of the batch kernel) and the
    DataLoader path both train one epoch and evaluate."""
    _fake_cifar_bin(tmp_path / "data")
    for mode in ("1", "0"):
        out = _run([sys.executable, "pytorch/resnet/main.py", "--device", "cpu", "--backend", "gloo", "--workers", "0",
                    "--num_epochs", "1", "--batch_size", "8", "--data_root", str(tmp_path / "data"),
                    "--data_on_device", mode, "--model_dir", str(tmp_path / mode)])
        assert "Epoch: 0, Accuracy:" in out and "Epoch 0 completed" in out


def test_unet_device_cached_data(tmp_path):
    out = _run([sys.executable, "pytorch/unet/train.py", *COMMON, "--num_epochs", "1", "--batch_size", "2",
                "--image_size", "32", "--synthetic_size", "6", "--eval_every", "1", "--data_on_device", "1",
                "--log_dir", str(tmp_path / "logs"), "--model_dir", str(tmp_path)])
    assert "Dice Score" in out and "TRAINING COMPLETED" in out
