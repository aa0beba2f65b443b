"""ResNet DDP trainer, variant A (reference: pytorch/resnet/main.py -- batch 128, per-step loss).
Same flags and defaults; launch with mpirun or torchrun.  See deeplearning_mpi_amd/apps/classification.py."""
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))

from deeplearning_mpi_amd.apps.classification import main  # noqa: E402

if __name__ == "__main__":
    main("main")
