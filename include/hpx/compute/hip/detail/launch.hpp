// hpx/compute/hip/detail/launch.hpp -- launch an arbitrary device closure on a
// target's stream, the HIP counterpart of hpx/compute/cuda/detail/launch.hpp:32-137.
//
// The reference instantiates `launch_function<Closure>` per closure and runs it
// with <<<grid, block, 0, stream>>>.  That needs the user's translation unit to
// be compiled by a device compiler: here hipcc (__HIPCC__).  A TU built with a
// plain host compiler gets the C-ABI path only (the built-in functors of
// <hpx/compute/hip/functional.hpp>); asking it to launch a closure is a
// compile-time error, never a silent host fallback.
//
// HPX_HOST_DEVICE / HPX_DEVICE: <hpx/config/compiler_specific.hpp>.
#pragma once

#include <hpx/compute/hip.hpp>

#include <cstddef>
#include <cstdint>
#include <tuple>
#include <type_traits>
#include <utility>

#include <hpx/config/compiler_specific.hpp>

namespace hpx { namespace compute { namespace hip { namespace detail {

template <typename...>
constexpr bool dependent_false = false;

#if HPX_HAVE_HIP_DEVICE_CLOSURES
// launch.hpp:32-36
template <typename Closure>
__global__ void launch_function(Closure closure) {
    closure();
}

// An aggregate argument pack (std::tuple is not trivially copyable, kernel
// arguments must be).
template <typename... Ts>
struct arg_pack {};
template <typename T, typename... Ts>
struct arg_pack<T, Ts...> {
    T head;
    arg_pack<Ts...> tail;
};
template <std::size_t I, typename T, typename... Ts>
__host__ __device__ auto& pack_get(arg_pack<T, Ts...>& p) {
    if constexpr (I == 0) return p.head;
    else return pack_get<I - 1>(p.tail);
}
inline arg_pack<> make_pack() { return {}; }
template <typename T, typename... Ts>
arg_pack<std::decay_t<T>, std::decay_t<Ts>...> make_pack(T&& t, Ts&&... ts) {
    return {std::forward<T>(t), make_pack(std::forward<Ts>(ts)...)};
}

// launch.hpp:38-70: the function object plus its bound arguments, by value.
template <typename F, typename... Ts>
struct closure {
    F f;
    arg_pack<Ts...> args;

    template <std::size_t... I>
    __device__ void call(std::index_sequence<I...>) {
        f(pack_get<I>(args)...);
    }
    __device__ void operator()() { call(std::index_sequence_for<Ts...>{}); }
};

// launch.hpp:129-137: no device synchronisation; errors -> kernel_error.
template <typename F, typename... Ts>
void launch(hip::target const& t, dim3 grid, dim3 block, F&& f, Ts&&... ts) {
    using C = closure<std::decay_t<F>, std::decay_t<Ts>...>;
    static_assert(std::is_trivially_copyable<C>::value,
                  "a device closure and its arguments must be trivially copyable (kernel arguments)");
    static_assert(sizeof(C) <= 4096, "device closure larger than the kernel argument segment");
    C c{std::forward<F>(f), make_pack(std::forward<Ts>(ts)...)};
    if (grid.x == 0 || block.x == 0) return;
    hipLaunchKernelGGL(launch_function<C>, grid, block, 0, reinterpret_cast<hipStream_t>(t.stream()), c);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess)
        throw kernel_error(static_cast<int>(e), std::string("hip::detail::launch: ") + hipGetErrorString(e));
}

// Grid for a flat 1-D launch over n work items: 256-thread blocks, enough
// blocks to cover n once up to 32 per CU (256 CUs), grid-stride beyond.
inline dim3 flat_grid(uint64_t n, unsigned block = 256) {
    uint64_t blocks = (n + block - 1) / block;
    const uint64_t cap = 256u * 32u;
    return dim3(static_cast<unsigned>(blocks < cap ? blocks : cap));
}
#else
template <typename F, typename... Ts>
void launch(hip::target const&, unsigned, unsigned, F&&, Ts&&...) {
    static_assert(dependent_false<F>,
                  "launching a device closure needs the translation unit to be compiled by hipcc "
                  "(HPX_HOST_DEVICE lambdas); with a host compiler use the functors of "
                  "<hpx/compute/hip/functional.hpp>");
}
#endif

}}}}  // namespace hpx::compute::hip::detail
