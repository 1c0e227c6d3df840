// hpx/dataflow.hpp -- hpx::dataflow (forwarding header, as in HPX 1.4.0)
#pragma once
#include <hpx/lcos/dataflow.hpp>
