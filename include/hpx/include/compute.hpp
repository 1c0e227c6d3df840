// hpx/include/compute.hpp -- HIP counterpart of the reference's compute umbrella
// (hpx/include/compute.hpp: target, allocator, executors, vector).
#pragma once
#include <hpx/compute/hip.hpp>
#include <hpx/compute/hip/concurrent_executor.hpp>
#include <hpx/compute/hip/default_executor.hpp>
#include <hpx/compute/hip/functional.hpp>
