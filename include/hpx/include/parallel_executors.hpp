// hpx/include/parallel_executors.hpp -- forwards to the HIP backend's algorithm layer.
#pragma once
#include <hpx/parallel/algorithms.hpp>
