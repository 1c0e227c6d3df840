// hpx/include/partitioned_vector.hpp -- hpx::partitioned_vector over HIP
// targets and its segmented algorithms (the reference's umbrella of the
// same name, hpx/include/partitioned_vector.hpp).
#pragma once
#include <hpx/components/containers/partitioned_vector/partitioned_vector.hpp>
#include <hpx/parallel/algorithms.hpp>
