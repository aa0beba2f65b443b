"""deeplearning_mpi_amd -- an MI355X-native (gfx950 / CDNA4) MPI-launched data-parallel training
framework with the capabilities of unlikeghost/DeepLearning-MPI.

Layers (bottom-up): native kernels + RCCL comm + reducer (``_C``), MPI bootstrap (``_mpi``),
compute backends (``ops``), parameter arena (``utils.arena``), engine models (``models``),
distributed runtime (``parallel``), fused optimizers (``optim``), data (``data``).
"""
__version__ = "0.1.0"

from . import ops, models, parallel, optim, data, utils  # noqa: E402,F401
from .parallel import DistributedDataParallel, init_distributed, get_comm, destroy_distributed  # noqa: E402,F401
