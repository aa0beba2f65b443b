"""CIFAR-10 preparation (reference: pytorch/resnet/download.py, which downloads via torchvision).

This framework never reaches the network from training processes (downloading is not
multi-process safe, reference main.py:89-91).  Place the official CIFAR-10 binary release
(cifar-10-batches-bin/) or python release (cifar-10-batches-py/) under ./data; this script
verifies it, or extracts a local cifar-10-*.tar.gz archive if one is present."""
import glob
import os
import sys
import tarfile

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))

root = "./data"
os.makedirs(root, exist_ok=True)
for arc in glob.glob(os.path.join(root, "cifar-10-*.tar.gz")):
    with tarfile.open(arc) as t:
        t.extractall(root, filter="data")
from deeplearning_mpi_amd.data import CIFAR10  # noqa: E402

try:
    tr, te = CIFAR10(root, train=True), CIFAR10(root, train=False)
    print(f"CIFAR-10 ready: {len(tr)} train / {len(te)} test images")
except FileNotFoundError as e:
    print(e)
    print("Copy the CIFAR-10 archive (cifar-10-binary.tar.gz or cifar-10-python.tar.gz) into ./data and rerun.")
    sys.exit(1)
