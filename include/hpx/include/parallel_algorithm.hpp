// hpx/include/parallel_algorithm.hpp -- forwards to the HIP backend's algorithm layer.
#pragma once
#include <hpx/parallel/algorithms.hpp>
