// hpx/include/lcos.hpp -- futures and their composition (hpx/include/lcos.hpp)
#pragma once
#include <hpx/lcos/async.hpp>
#include <hpx/lcos/dataflow.hpp>
#include <hpx/lcos/future.hpp>
#include <hpx/lcos/local/sliding_semaphore.hpp>
#include <hpx/lcos/when_all.hpp>
#include <hpx/util/unwrapping.hpp>
