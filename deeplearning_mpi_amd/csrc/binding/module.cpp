// Python module `deeplearning_mpi_amd._C`: gfx950 kernels + RCCL comm + DDP reducer.
#include <torch/extension.h>

#include "comm.h"
#include "ops.h"

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "MI355X-native kernels, RCCL communicator and gradient-bucket reducer";
  dlmpi_ext::register_ops(m);
  dlmpi_ext::register_comm(m);
  m.attr("ARCH") = "gfx950";
}
