// hpx/include/parallel_for_each.hpp -- forwards to the HIP backend's algorithm layer.
#pragma once
#include <hpx/parallel/algorithms.hpp>
