#pragma once
#include <torch/extension.h>

namespace amd {

// Registers the `Reducer` class (DDP bucketed all-reduce core) on module `m`.
void register_reducer(pybind11::module_& m);

}  // namespace amd
