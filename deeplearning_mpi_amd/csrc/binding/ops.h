#pragma once
#include <torch/extension.h>

namespace dlmpi_ext {
void register_ops(pybind11::module& m);
// launch the queued (deferred) weight-gradient split reductions on the current stream (ops.cpp)
void wgrad_flush();
}
