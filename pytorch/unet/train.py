"""UNet DDP trainer (reference: pytorch/unet/train.py).  Same flags, defaults and log format;
launch with mpirun or torchrun (see run.sh).  Implementation: deeplearning_mpi_amd/apps/segmentation.py."""
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))

from deeplearning_mpi_amd.apps.segmentation import main  # noqa: E402

if __name__ == "__main__":
    main()
