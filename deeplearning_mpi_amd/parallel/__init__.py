from .bootstrap import LaunchInfo, detect_launcher  # noqa: F401
from .comm import (Communicator, MPICommunicator, RcclCommunicator, SingleCommunicator,  # noqa: F401
                   TorchCommunicator, destroy_distributed, get_comm, init_distributed)
from .ddp import DistributedDataParallel  # noqa: F401
