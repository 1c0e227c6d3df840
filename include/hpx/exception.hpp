// hpx/exception.hpp -- the error types of the MI355X backend's C++ layer.
//
//   hpx::exception      <- hpx/exception.hpp (HPX's exception with an error
//                          code; here the code is the C ABI status: a
//                          hipError_t value or an HPXHIP_ERROR_* code)
//   hpx::kernel_error   <- the error of a failed launch or a device-side
//                          failure (cuda/detail/launch.hpp:106-113)
//   hpx::out_of_memory  <- an allocation failure, a std::bad_alloc as the
//                          reference's allocator throws (cuda/allocator.hpp:118-124)
//
// Parallel algorithms never let these escape directly: every non-bad_alloc
// failure reaches the caller wrapped in hpx::exception_list
// (<hpx/exception_list.hpp>).
#pragma once

#include <hpxhip.h>

#include <new>
#include <stdexcept>
#include <string>
#include <utility>

namespace hpx {

struct exception : std::runtime_error {
    int status;
    exception(int s, std::string const& what) : std::runtime_error(what), status(s) {}
};
struct kernel_error : exception {
    using exception::exception;
};
struct out_of_memory : std::bad_alloc {
    std::string msg;
    explicit out_of_memory(std::string m) : msg(std::move(m)) {}
    const char* what() const noexcept override { return msg.c_str(); }
};

}  // namespace hpx
