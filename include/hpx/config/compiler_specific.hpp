// hpx/config/compiler_specific.hpp -- HPX_HOST_DEVICE / HPX_DEVICE as in
// libs/config/include/hpx/config/compiler_specific.hpp:95-126: host+device
// when the translation unit is compiled by hipcc (then the algorithms can
// instantiate kernels for the caller's function objects,
// HPX_HAVE_HIP_DEVICE_CLOSURES = 1), plain host functions otherwise.
#pragma once

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#ifndef HPX_HOST_DEVICE
#define HPX_HOST_DEVICE __host__ __device__
#endif
#ifndef HPX_DEVICE
#define HPX_DEVICE __device__
#endif
#define HPX_HAVE_HIP_DEVICE_CLOSURES 1
#else
#ifndef HPX_HOST_DEVICE
#define HPX_HOST_DEVICE
#endif
#ifndef HPX_DEVICE
#define HPX_DEVICE
#endif
#define HPX_HAVE_HIP_DEVICE_CLOSURES 0
#endif
