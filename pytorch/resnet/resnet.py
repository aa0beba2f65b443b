"""ResNet DDP trainer, variant B (reference: pytorch/resnet/resnet.py -- batch 32, 8 workers,
eval/save before training on eval epochs, test batch 128).  See deeplearning_mpi_amd/apps/classification.py."""
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))

from deeplearning_mpi_amd.apps.classification import main  # noqa: E402

if __name__ == "__main__":
    main("resnet")
