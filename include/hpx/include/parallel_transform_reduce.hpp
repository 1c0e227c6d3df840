// hpx/include/parallel_transform_reduce.hpp -- forwards to the HIP backend's algorithm layer.
#pragma once
#include <hpx/parallel/algorithms.hpp>
