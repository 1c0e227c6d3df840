// hpx/hpx.hpp -- umbrella header of the HIP backend's HPX mirror.
#pragma once
#include <hpx/include/compute.hpp>
#include <hpx/include/lcos.hpp>
#include <hpx/include/partitioned_vector.hpp>
#include <hpx/parallel/algorithms.hpp>
#include <hpx/parallel/execution.hpp>
#include <hpx/parallel/heat_solver.hpp>
