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

// A reduction of a generic for_loop body (for_loop_reduction.hpp:35-132):
// every thread folds into a private view that starts at the identity, the
// views are combined per block in a fixed tree and the block partials in
// block order, and the loop exit folds the result into the live-out variable.
template <typename T, typename Op>
struct red_arg {
    T id;
    Op op;
};
template <typename A>
struct is_red_arg : std::false_type {};
template <typename T, typename Op>
struct is_red_arg<red_arg<T, Op>> : std::true_type {};
// position of reduction I among the loop's reductions
template <std::size_t I, typename... A>
constexpr std::size_t red_ordinal() {
    constexpr bool r[] = {is_red_arg<A>::value..., false};
    std::size_t k = 0;
    for (std::size_t j = 0; j < I; ++j) k += r[j] ? 1 : 0;
    return k;
}
constexpr int kLoopReduceThreads = 256;
constexpr unsigned kLoopReduceMaxBlocks = 1024;

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
// ---- generic for_loop bodies with reductions
template <typename A>
struct view_of {
    using type = uint64_t;  // unused slot for a loop variable
};
template <typename T, typename Op>
struct view_of<red_arg<T, Op>> {
    using type = T;
};
template <typename T>
__device__ T* loop_arg(strided_ptr<T>& v, uint64_t&, uint64_t i) {
    return v.p + static_cast<int64_t>(i) * v.stride;
}
template <typename T, typename Op>
__device__ T& loop_arg(red_arg<T, Op>&, T& view, uint64_t) {
    return view;
}
template <typename A, typename V>
__device__ void init_view(A const&, V&) {}
template <typename T, typename Op>
__device__ void init_view(red_arg<T, Op> const& r, T& view) {
    view = r.id;
}

// Pass 1: grid-stride loop calling f(args at i...), then per reduction a
// fixed LDS tree over the block's views -> partials[block][ordinal].
template <typename F, typename... A, std::size_t... I>
__device__ void loop_reduce_block(F& f, uint64_t n, compute::hip::detail::arg_pack<A...>& args,
                                  compute::hip::detail::arg_pack<typename view_of<A>::type...>& views,
                                  uint64_t* partials, unsigned nred, std::index_sequence<I...>) {
    using compute::hip::detail::pack_get;
    (init_view(pack_get<I>(args), pack_get<I>(views)), ...);
    for (uint64_t i = first_index(); i < n; i += grid_stride())
        f(loop_arg(pack_get<I>(args), pack_get<I>(views), i)...);
    __shared__ uint64_t s_bits[kLoopReduceThreads];
    auto reduce_one = [&](auto& r, auto& view, std::size_t ord) {
        using T = std::decay_t<decltype(view)>;
        static_assert(sizeof(T) <= 8 && std::is_trivially_copyable<T>::value,
                      "for_loop: reduction values of up to 8 trivially copyable bytes");
        T* s = reinterpret_cast<T*>(s_bits);
        __syncthreads();
        s[threadIdx.x] = view;
        __syncthreads();
        for (unsigned w = kLoopReduceThreads / 2; w > 0; w /= 2) {
            if (threadIdx.x < w) s[threadIdx.x] = r.op(s[threadIdx.x], s[threadIdx.x + w]);
            __syncthreads();
        }
        if (threadIdx.x == 0) {
            uint64_t bits = 0;
            __builtin_memcpy(&bits, &s[0], sizeof(T));
            partials[static_cast<uint64_t>(blockIdx.x) * nred + ord] = bits;
        }
    };
    (
        [&] {
            if constexpr (is_red_arg<A>::value)
                reduce_one(pack_get<I>(args), pack_get<I>(views), red_ordinal<I, A...>());
        }(),
        ...);
}
template <typename F, typename... A>
__global__ __launch_bounds__(kLoopReduceThreads) void k_loop_reduce(F f, uint64_t n,
                                                                    compute::hip::detail::arg_pack<A...> args,
                                                                    uint64_t* partials, unsigned nred) {
    compute::hip::detail::arg_pack<typename view_of<A>::type...> views{};
    loop_reduce_block(f, n, args, views, partials, nred, std::index_sequence_for<A...>{});
}
// Pass 2 (one thread per reduction): the block partials in block order,
// starting from the identity -> out[ordinal] (8-byte words).
template <typename... A, std::size_t... I>
__device__ void loop_reduce_fold_all(compute::hip::detail::arg_pack<A...>& args, uint64_t const* partials,
                                     unsigned nblocks, unsigned nred, uint64_t* out, std::index_sequence<I...>) {
    using compute::hip::detail::pack_get;
    (
        [&] {
            if constexpr (is_red_arg<A>::value) {
                constexpr std::size_t ord = red_ordinal<I, A...>();
                if (threadIdx.x == ord) {
                    auto& r = pack_get<I>(args);
                    using T = std::decay_t<decltype(r.id)>;
                    T acc = r.id;
                    for (unsigned b = 0; b < nblocks; ++b) {
                        T x;
                        __builtin_memcpy(&x, &partials[static_cast<uint64_t>(b) * nred + ord], sizeof(T));
                        acc = r.op(acc, x);
                    }
                    uint64_t bits = 0;
                    __builtin_memcpy(&bits, &acc, sizeof(T));
                    out[ord] = bits;
                }
            }
        }(),
        ...);
}
template <typename... A>
__global__ void k_loop_reduce_fold(compute::hip::detail::arg_pack<A...> args, uint64_t const* partials,
                                   unsigned nblocks, unsigned nred, uint64_t* out) {
    loop_reduce_fold_all(args, partials, nblocks, nred, out, std::index_sequence_for<A...>{});
}
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

// A generic for_loop body with reductions: args are strided_ptr (loop
// iterator, inductions) and red_arg (reductions) in call order; the
// reductions' results land as 8-byte words in out[0..nred) (device).
// `partials` holds kLoopReduceMaxBlocks * nred words.
template <typename F, typename... A>
void device_loop_reduce(compute::hip::target const& t, F const& f, uint64_t n, uint64_t* partials, uint64_t* out,
                        A const&... a) {
#if HPX_HAVE_HIP_DEVICE_CLOSURES
    constexpr unsigned nred = static_cast<unsigned>((0u + ... + (is_red_arg<A>::value ? 1u : 0u)));
    static_assert(nred >= 1 && nred <= 8, "for_loop: one to eight reductions (their results share one slot)");
    const dim3 g = compute::hip::detail::flat_grid(n);
    const unsigned nb = n == 0 ? 1u : (g.x < kLoopReduceMaxBlocks ? g.x : kLoopReduceMaxBlocks);
    auto args = compute::hip::detail::make_pack(a...);
    static_assert(std::is_trivially_copyable<decltype(args)>::value && std::is_trivially_copyable<F>::value,
                  "a for_loop body and its reductions must be trivially copyable (kernel arguments)");
    const hipStream_t s = reinterpret_cast<hipStream_t>(t.stream());
    hipLaunchKernelGGL((closures::k_loop_reduce<F, A...>), dim3(nb), dim3(kLoopReduceThreads), 0, s, f, n, args,
                       partials, nred);
    hipLaunchKernelGGL((closures::k_loop_reduce_fold<A...>), dim3(1), dim3(64), 0, s, args,
                       static_cast<uint64_t const*>(partials), nb, nred, out);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) compute::hip::detail::check(static_cast<int>(e), "for_loop (device closure with reductions)");
#else
    static_assert(compute::hip::detail::dependent_false<F>,
                  "for_loop: a loop body with reductions is a functional::loop_accumulate(_all), or the translation "
                  "unit is compiled with hipcc");
    (void)t, (void)f, (void)n, (void)partials, (void)out;
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
