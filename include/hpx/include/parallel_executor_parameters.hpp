// hpx/include/parallel_executor_parameters.hpp -- forwards to the HIP backend's algorithm layer.
#pragma once
#include <hpx/parallel/algorithms.hpp>
