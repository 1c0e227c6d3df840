// hpx/parallel/detail/device_closures.hpp -- the algorithms' path for
// arbitrary HPX_HOST_DEVICE function objects, used when the calling
// translation unit is compiled by hipcc.
//
// The reference runs every GPU algorithm by instantiating its generic
// launch_function<Closure> with the user's callable
// (hpx/compute/cuda/detail/launch.hpp:32-137, default_executor.hpp:87-136):
// for_each / transform / for_loop with lambdas are the whole GPU test surface
// (tests/unit/computeapi/cuda/{for_each,transform,for_loop}_compute.cu).  A
// precompiled C ABI cannot take closures, so these bodies are header
// templates instantiated per callable by hipcc: flat grid-stride kernels with
// 64-bit indices (the reference's thread-per-element grid uses int math,
// default_executor.hpp:52-55,109-121).  A host-compiled TU that passes a
// callable without a device mapping gets a static_assert naming both ways
// out, never a host fallback.
#pragma once

#include <hpx/compute/hip.hpp>
#include <hpx/compute/hip/detail/launch.hpp>

#include <cstdint>
#include <type_traits>
#include <utility>

namespace hpx { namespace parallel { inline namespace v1 { namespace detail {

// A loop variable of a generic for_loop body: raw device pointer + stride
// (for_loop_induction.hpp:210-219: value at iteration i = base + stride * i).
template <typename T>
struct strided_ptr {
    T* p;
    int64_t stride;
};

#if HPX_HAVE_HIP_DEVICE_CLOSURES
namespace closures {
__device__ inline uint64_t first_index() { return uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; }
__device__ inline uint64_t grid_stride() { return uint64_t(gridDim.x) * blockDim.x; }

struct for_each_body {  // for_each.hpp:48-123: f(*it)
    template <typename F, typename T>
    __device__ void operator()(F& f, T* p, uint64_t n) const {
        for (uint64_t i = first_index(); i < n; i += grid_stride()) f(p[i]);
    }
};
struct transform_body {  // transform.hpp:67-136: *dest = f(*it)
    template <typename F, typename TI, typename TO>
    __device__ void operator()(F& f, TI const* in, TO* out, uint64_t n) const {
        for (uint64_t i = first_index(); i < n; i += grid_stride()) out[i] = f(in[i]);
    }
};
struct transform2_body {  // transform.hpp:340-408: *dest = f(*it1, *it2)
    template <typename F, typename T1, typename T2, typename TO>
    __device__ void operator()(F& f, T1 const* a, T2 const* b, TO* out, uint64_t n) const {
        for (uint64_t i = first_index(); i < n; i += grid_stride()) out[i] = f(a[i], b[i]);
    }
};
struct loop_body {  // for_loop.hpp:60-120: f(first + i*stride, inductions...)
    template <typename F, typename... Ts>
    __device__ void operator()(F& f, uint64_t n, strided_ptr<Ts>&... v) const {
        for (uint64_t i = first_index(); i < n; i += grid_stride())
            f((v.p + static_cast<int64_t>(i) * v.stride)...);
    }
};
}  // namespace closures
#endif

template <typename F, typename T>
void device_for_each(compute::hip::target const& t, F const& f, T* p, uint64_t n) {
#if HPX_HAVE_HIP_DEVICE_CLOSURES
    compute::hip::detail::launch(t, compute::hip::detail::flat_grid(n), dim3(256), closures::for_each_body{}, f, p, n);
#else
    static_assert(compute::hip::detail::dependent_false<F>,
                  "for_each: this function object has no device mapping -- specialise "
                  "hpx::compute::hip::traits::unary<F>, or compile the translation unit with hipcc");
    (void)t, (void)f, (void)p, (void)n;
#endif
}

template <typename F, typename TI, typename TO>
void device_transform(compute::hip::target const& t, F const& f, TI const* in, TO* out, uint64_t n) {
#if HPX_HAVE_HIP_DEVICE_CLOSURES
    compute::hip::detail::launch(t, compute::hip::detail::flat_grid(n), dim3(256), closures::transform_body{}, f, in,
                                 out, n);
#else
    static_assert(compute::hip::detail::dependent_false<F>,
                  "transform: this function object has no device mapping -- specialise "
                  "hpx::compute::hip::traits::unary<F>, or compile the translation unit with hipcc");
    (void)t, (void)f, (void)in, (void)out, (void)n;
#endif
}

template <typename F, typename T1, typename T2, typename TO>
void device_transform2(compute::hip::target const& t, F const& f, T1 const* a, T2 const* b, TO* out, uint64_t n) {
#if HPX_HAVE_HIP_DEVICE_CLOSURES
    compute::hip::detail::launch(t, compute::hip::detail::flat_grid(n), dim3(256), closures::transform2_body{}, f, a,
                                 b, out, n);
#else
    static_assert(compute::hip::detail::dependent_false<F>,
                  "transform: this function object has no device mapping -- specialise "
                  "hpx::compute::hip::traits::binary<F>, or compile the translation unit with hipcc");
    (void)t, (void)f, (void)a, (void)b, (void)out, (void)n;
#endif
}

template <typename F, typename... Ts>
void device_loop(compute::hip::target const& t, F const& f, uint64_t n, strided_ptr<Ts>... v) {
#if HPX_HAVE_HIP_DEVICE_CLOSURES
    compute::hip::detail::launch(t, compute::hip::detail::flat_grid(n), dim3(256), closures::loop_body{}, f, n, v...);
#else
    static_assert(compute::hip::detail::dependent_false<F>,
                  "for_loop: this loop body is neither a functional::loop_assign/loop_accumulate nor compiled "
                  "by hipcc -- arbitrary loop bodies need the translation unit to be compiled with hipcc");
    (void)t, (void)f, (void)n;
#endif
}

}}}}  // namespace hpx::parallel::v1::detail
