#pragma once
#include <torch/extension.h>

namespace dlmpi_ext {
void register_ops(pybind11::module& m);
}
