// hpx/parallel/detail/device_algorithms.hpp -- reduce / transform_reduce,
// the scans, copy_if and sort with ARBITRARY HPX_HOST_DEVICE callables, when
// the calling translation unit is compiled by hipcc.
//
// The reference accepts any conv / op / pred / comp (transform_reduce.hpp:254,
// inclusive_scan.hpp:288-606, copy.hpp:585, sort.hpp:364 with a projection).
// The library's precompiled entry points take an operator KIND, so a function
// object with a traits mapping goes there (algorithms.hpp); anything else
// lands here and instantiates the library's OWN kernel bodies with the
// caller's callable (include/hpxhip/kernels/):
//
//   reduce / transform_reduce  reduce_kernel.hpp   (128-KiB blocks, DPP tree,
//                                                   fixed-order partial fold)
//   scans                      scan_kernel.hpp     (single pass, decoupled
//                                                   look-back, 16-B tiles)
//   copy_if                    copy_if_kernel.hpp  (ballot ranks, look-back)
//   sort (comp, proj)          merge_kernel.hpp    (block sort in LDS, then
//                                                   merge-path passes)
//
// A user operator has no known identity, but every GPU tree and scan pads its
// inactive lanes with one: such an op is lifted to opt<T> (a value or "none",
// "none" being the identity; common.hpp lifted_op).  A built-in operator
// (std::plus, ...) with a user conv keeps the plain value type.
//
// Semantics: reduce / transform_reduce need an associative and commutative
// op (reduce.hpp: "the behavior is non-deterministic if binary_op is not
// associative or not commutative"); the scans need associativity only (the
// kernels combine in index order); copy_if is stable; the merge sort is
// stable (a valid std::sort order, ties in input order).
#pragma once

#include <hpx/compute/hip.hpp>
#include <hpx/compute/hip/detail/launch.hpp>
#include <hpx/compute/hip/functional.hpp>

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <type_traits>
#include <utility>

#if HPX_HAVE_HIP_DEVICE_CLOSURES
#include <hpxhip/kernels/copy_if_kernel.hpp>
#include <hpxhip/kernels/merge_kernel.hpp>
#include <hpxhip/kernels/reduce_kernel.hpp>
#include <hpxhip/kernels/scan_kernel.hpp>
#endif

namespace hpx { namespace parallel { inline namespace v1 { namespace detail {
namespace dev {

#if HPX_HAVE_HIP_DEVICE_CLOSURES
namespace K = ::hpxhip;
namespace tr = hpx::compute::hip::traits;

// built-in operator kinds -> the kernels' device functors (identity known)
template <int Kind> struct kind_op;
template <> struct kind_op<HPXHIP_PLUS> { using type = K::op_plus; };
template <> struct kind_op<HPXHIP_MULTIPLIES> { using type = K::op_multiplies; };
template <> struct kind_op<HPXHIP_MIN> { using type = K::op_min; };
template <> struct kind_op<HPXHIP_MAX> { using type = K::op_max; };
template <> struct kind_op<HPXHIP_BIT_AND> { using type = K::op_bit_and; };
template <> struct kind_op<HPXHIP_BIT_OR> { using type = K::op_bit_or; };
template <> struct kind_op<HPXHIP_BIT_XOR> { using type = K::op_bit_xor; };
template <typename Op>
using builtin_op_t = typename kind_op<tr::binop_t<Op>::kind>::type;
// the device operator of Op: its built-in functor, or Op lifted to opt<T>
template <typename Op, bool BUILTIN = tr::is_binop<Op>>
struct dev_op {
    using type = K::lifted_op<std::decay_t<Op>>;
};
template <typename Op>
struct dev_op<Op, true> {
    using type = builtin_op_t<Op>;
};

// the scans' device operator: a built-in kind, or the user operator without
// an identity (K::noid_op)
template <typename Op, bool = tr::is_binop<Op>>
struct scan_op {
    using type = K::noid_op<std::decay_t<Op>>;
};
template <typename Op>
struct scan_op<Op, true> {
    using type = builtin_op_t<Op>;
};

inline hipStream_t stream_of(compute::hip::target const& t) { return reinterpret_cast<hipStream_t>(t.stream()); }

inline void* scratch(compute::hip::target const& t, std::size_t bytes, char const* what) {
    void* p = nullptr;
    compute::hip::detail::check(hpxhip_stream_scratch(t.stream(), bytes, &p), what);
    return p;
}
inline uint32_t* error_word(compute::hip::target const& t) {
    uint32_t* w = nullptr;
    compute::hip::detail::check(hpxhip_device_error_word(t.stream(), &w), "device error word");
    return w;
}
inline void launched(char const* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) throw hpx::kernel_error(static_cast<int>(e), std::string(what) + ": " +
                                                                                 hipGetErrorString(e));
}

// ------------------------------------------------------------------ reduce
// Element sources of reduce_kernel.hpp: conv on one / two elements, plain
// (built-in op) or lifted to opt<TA> (user op).
template <typename TI, typename TA, typename Conv, bool LIFT>
struct source1 {
    const TI* a;
    const TI* b;
    Conv conv;
    using R = std::conditional_t<LIFT, K::opt<TA>, TA>;
    __device__ __forceinline__ R elem(TI x) const {
        if constexpr (LIFT) return R{static_cast<TA>(conv(x)), 1u};
        else return static_cast<TA>(conv(x));
    }
};
template <typename TI, typename TA, typename Comb, bool LIFT>
struct source2 {
    const TI* a;
    const TI* b;
    Comb comb;
    using R = std::conditional_t<LIFT, K::opt<TA>, TA>;
    __device__ __forceinline__ R elem(TI x, TI y) const {
        if constexpr (LIFT) return R{static_cast<TA>(comb(x, y)), 1u};
        else return static_cast<TA>(comb(x, y));
    }
};

// *out_dev (a result slot) <- init (red) conv(x_0) (red) ...; the TA value
// sits at the start of the slot in both forms (opt<TA>::v is its first member).
template <typename TA, bool BINARY, typename TI, typename Red, typename Conv>
void reduce(compute::hip::target const& t, TI const* a, TI const* b, uint64_t n, TA init, Red const& red,
            Conv const& conv, void* out_dev) {
    constexpr bool lift = !tr::is_binop<Red>;
    using X = std::conditional_t<lift, K::opt<TA>, TA>;
    using Src = std::conditional_t<BINARY, source2<TI, TA, std::decay_t<Conv>, lift>,
                                   source1<TI, TA, std::decay_t<Conv>, lift>>;
    static_assert(sizeof(X) <= compute::hip::detail::device_pool::kSlotBytes, "reduce: result larger than a slot");
    X* partials = n ? static_cast<X*>(scratch(t, K::reduce_detail::max_blocks(n) * sizeof(X), "reduce scratch"))
                    : nullptr;
    Src src{a, b, conv};
    hipError_t e;
    if constexpr (lift) {
        using Op = K::lifted_op<std::decay_t<Red>>;
        e = K::reduce_detail::launch<TI, X, Src, Op, BINARY>(src, n, Op{red}, X{init, 1u}, static_cast<X*>(out_dev),
                                                             partials, stream_of(t));
    } else {
        using Op = builtin_op_t<Red>;
        e = K::reduce_detail::launch<TI, X, Src, Op, BINARY>(src, n, Op{}, init, static_cast<X*>(out_dev), partials,
                                                             stream_of(t));
    }
    if (e != hipSuccess) throw hpx::kernel_error(static_cast<int>(e), "transform_reduce (device closure)");
}

// -------------------------------------------------------------------- scans
template <typename V, typename X, typename Conv>
struct scan_conv {
    Conv conv;
    __device__ __forceinline__ X operator()(V x) const {
        if constexpr (std::is_same<X, V>::value) return static_cast<V>(conv(x));
        else return X{static_cast<V>(conv(x)), 1u};
    }
};

template <typename V, typename X, typename Cv, typename Op, bool INCL, bool ALIGNED>
void scan_launch(compute::hip::target const& t, V const* in, V* out, uint64_t n, Cv cv, Op op, X init) {
    namespace S = K::scan_detail;
    // a user operator scans plain values (noid_op, no identity needed): the
    // built-in kinds' tile shape, except 14 rounds for aligned 8-byte
    // integers (the identity-free wave scan's selects: 16 rounds spill 12
    // VGPRs, 14 fit in 120)
    constexpr bool noid = K::is_noid_op<Op>::value;
    constexpr int R = (noid && ALIGNED && sizeof(V) == 8 && std::is_integral<V>::value) ? 14
                                                                                           : S::rounds_for<V, ALIGNED>();
    constexpr uint64_t tile = S::tile_elems<V, R>();
    const uint64_t ntiles = (n + tile - 1) / tile;
    const std::size_t state = (256 + ntiles * K::tile_state<X>::bytes_per_tile() + 255) / 256 * 256;
    char* ws = static_cast<char*>(scratch(t, state, "scan scratch"));
    compute::hip::detail::check(hpxhip_memset_async(ws, 0, state, t.stream()), "scan scratch");
    K::scan_detail::scan_state<X> st{reinterpret_cast<uint64_t*>(ws + 256), error_word(t)};
    hipLaunchKernelGGL((S::k_scan<V, Cv, Op, INCL, ALIGNED, R, S::kThreads, true, 1, false, 1, false, true, X>),
                       dim3(static_cast<unsigned>(ntiles)), dim3(S::kThreads), 0, stream_of(t), in, out, n, cv, op,
                       init, static_cast<X const*>(nullptr), reinterpret_cast<uint32_t*>(ws), st);
    launched("scan (device closure)");
}

template <typename V, typename Op, typename Conv, typename T>
void scan(compute::hip::target const& t, V const* in, V* out, uint64_t n, Op const& op, Conv const& conv, T init,
          bool inclusive) {
    static_assert(sizeof(V) == 4 || sizeof(V) == 8, "scan (device closure): 4- or 8-byte element types");
    if (n == 0) return;
    // A user operator has no known identity: round 3 lifted it to opt<V>
    // (flag + padding per element: 8 rounds instead of 16, 2^30 int64 3.43
    // vs 2.66 ms, profiles/r04_closure_timing_first.log); the kernel now runs
    // it on plain values with the identity-free scan (K::noid_op).
    constexpr bool lift = !tr::is_binop<Op>;
    using X = V;
    using Cv = scan_conv<V, X, std::decay_t<Conv>>;
    using OpD = typename scan_op<Op>::type;
    const OpD opd = [&] {
        if constexpr (lift) return OpD{op};
        else return OpD{};
    }();
    const X iv = static_cast<V>(init);
    const bool aligned = (reinterpret_cast<uintptr_t>(in) | reinterpret_cast<uintptr_t>(out)) % 16 == 0;
    Cv cv{conv};
    if (inclusive) {
        if (aligned) scan_launch<V, X, Cv, OpD, true, true>(t, in, out, n, cv, opd, iv);
        else scan_launch<V, X, Cv, OpD, true, false>(t, in, out, n, cv, opd, iv);
    } else {
        if (aligned) scan_launch<V, X, Cv, OpD, false, true>(t, in, out, n, cv, opd, iv);
        else scan_launch<V, X, Cv, OpD, false, false>(t, in, out, n, cv, opd, iv);
    }
}

// ------------------------------------------------------------------ copy_if
template <typename T, typename Pred>
struct as_bool_pred {
    Pred pred;
    __device__ __forceinline__ bool operator()(T x) const { return static_cast<bool>(pred(x)); }
};

template <typename T, typename P, bool ALIGNED, typename SV>
void copy_if_launch(compute::hip::target const& t, T const* in, T* out, uint64_t n, P p, uint64_t* count_dev) {
    namespace C = K::copy_if_detail;
    constexpr int R = 8;
    constexpr uint64_t tile = C::tile_elems<T, R>();
    const uint64_t ntiles = (n + tile - 1) / tile;
    const std::size_t state = (256 + ntiles * K::tile_state<SV>::bytes_per_tile() + 255) / 256 * 256;
    char* ws = static_cast<char*>(scratch(t, state, "copy_if scratch"));
    compute::hip::detail::check(hpxhip_memset_async(ws, 0, state, t.stream()), "copy_if scratch");
    K::tile_state<SV> st{reinterpret_cast<uint64_t*>(ws + 256), error_word(t)};
    if constexpr (ALIGNED) {
        // r05: the shipped pipelined form (copy_if.hip), one persistent
        // workgroup per CU
        static std::atomic<int> cus[64];
        const int dev = t.device();
        int c = dev >= 0 && dev < 64 ? cus[dev].load(std::memory_order_relaxed) : 0;
        if (c <= 0) {
            c = static_cast<int>(t.native_handle().processing_units());
            if (dev >= 0 && dev < 64) cus[dev].store(c, std::memory_order_relaxed);
        }
        const uint64_t grid = std::min<uint64_t>(ntiles, static_cast<uint64_t>(c));
        hipLaunchKernelGGL((C::k_copy_if_pipe<T, P, R, SV>), dim3(static_cast<unsigned>(grid)), dim3(C::kThreads), 0,
                           stream_of(t), in, out, n, p, count_dev, reinterpret_cast<uint32_t*>(ws), st, ntiles,
                           static_cast<const uint64_t*>(nullptr));
        launched("copy_if (device closure)");
        return;
    }
    // blockIdx tile order with the fixed-association look-back (the shipped
    // choice for copy_if, copy_if.hip); 4 waves per SIMD: a user predicate
    // may need more than 64 VGPRs.  r04: the shipped kernel's 8-byte
    // write-out (nt 16-B stores, 4 rounds per LDS batch) and one-hop
    // look-back took the lambda copy_if from 1.0x to 1.23x of the kind path
    // here (profiles/r04_closure_timing_copyif.log), so this form keeps them off.
    hipLaunchKernelGGL((C::k_copy_if<T, P, ALIGNED, R, 4, 0, SV, false, false, 1, true>),
                       dim3(static_cast<unsigned>(ntiles)),
                       dim3(C::kThreads), 0, stream_of(t), in, out, n, p, count_dev, reinterpret_cast<uint32_t*>(ws),
                       st, ntiles, static_cast<const uint64_t*>(nullptr));
    launched("copy_if (device closure)");
}

template <typename T, typename Pred>
void copy_if(compute::hip::target const& t, T const* in, T* out, uint64_t n, Pred const& pred, uint64_t* count_dev) {
    static_assert(16 % sizeof(T) == 0, "copy_if (device closure): element size must divide 16 bytes");
    using P = as_bool_pred<T, std::decay_t<Pred>>;
    if (n == 0) {
        compute::hip::detail::check(hpxhip_memset_async(count_dev, 0, sizeof(uint64_t), t.stream()), "copy_if count");
        return;
    }
    const bool aligned = reinterpret_cast<uintptr_t>(in) % 16 == 0;
    const bool small = n < (uint64_t{1} << 32);
    if (aligned && small) copy_if_launch<T, P, true, uint32_t>(t, in, out, n, P{pred}, count_dev);
    else if (aligned) copy_if_launch<T, P, true, uint64_t>(t, in, out, n, P{pred}, count_dev);
    else if (small) copy_if_launch<T, P, false, uint32_t>(t, in, out, n, P{pred}, count_dev);
    else copy_if_launch<T, P, false, uint64_t>(t, in, out, n, P{pred}, count_dev);
}

// --------------------------------------------------------------------- sort
// sort.hpp:364 -- comp(proj(a), proj(b)) (HPX_INVOKE of the projection).
template <typename T, typename Comp, typename Proj>
struct projected_less {
    Comp comp;
    Proj proj;
    __device__ __forceinline__ bool operator()(T const& a, T const& b) const {
        return static_cast<bool>(comp(proj(a), proj(b)));
    }
};

// Bottom-up merge sort: k_block_sort leaves sorted runs of kTile elements,
// then each pass merges run pairs (merge path) src -> dst, doubling the run
// width; the result is copied back if it ended in the scratch buffer.
template <typename T, typename Comp, typename Proj>
void merge_sort(compute::hip::target const& t, T* data, uint64_t n, Comp const& comp, Proj const& proj) {
    namespace M = K::merge_detail;
    if (n < 2) return;
    using L = projected_less<T, std::decay_t<Comp>, std::decay_t<Proj>>;
    const L less{comp, proj};
    const uint64_t ntiles = (n + M::kTile - 1) / M::kTile;
    hipLaunchKernelGGL((M::k_block_sort<T, L>), dim3(static_cast<unsigned>(ntiles)), dim3(M::kThreads), 0,
                       stream_of(t), data, n, less);
    launched("sort (device closure): block sort");
    if (ntiles == 1) return;
    const std::size_t buf = (n * sizeof(T) + 255) / 256 * 256;
    char* ws = static_cast<char*>(scratch(t, buf + (ntiles + 1) * sizeof(uint64_t), "sort scratch"));
    T* tmp = reinterpret_cast<T*>(ws);
    uint64_t* splits = reinterpret_cast<uint64_t*>(ws + buf);
    T* src = data;
    T* dst = tmp;
    // 16-B staging and stores when both buffers are 16-B aligned (the
    // scratch is; the data is unless the range starts inside a vector) and
    // n fills whole vectors (the staging reads whole vectors of each slice)
    const bool vec = reinterpret_cast<uintptr_t>(data) % 16 == 0 && reinterpret_cast<uintptr_t>(tmp) % 16 == 0 &&
                     n % M::vec_elems<T>() == 0;
    uint32_t* err = nullptr;  // a clamped split raises it (a caller racing the sort)
    compute::hip::detail::check(hpxhip_device_error_word(t.stream(), &err), "device error word");
    for (uint64_t w = M::kTile; w < n; w *= 2) {
        hipLaunchKernelGGL((M::k_pass_partition<T, L>), dim3(static_cast<unsigned>((ntiles + 255) / 256)), dim3(256),
                           0, stream_of(t), src, n, w, ntiles, less, splits);
        if (vec)
            hipLaunchKernelGGL((M::k_pass_merge<T, L, true>), dim3(static_cast<unsigned>(ntiles)), dim3(M::kThreads),
                               0, stream_of(t), src, n, w, splits, less, dst, err);
        else
            hipLaunchKernelGGL((M::k_pass_merge<T, L>), dim3(static_cast<unsigned>(ntiles)), dim3(M::kThreads), 0,
                               stream_of(t), src, n, w, splits, less, dst, err);
        launched("sort (device closure): merge pass");
        std::swap(src, dst);
    }
    if (src != data) compute::hip::detail::check(hpxhip_memcpy_async(data, src, n * sizeof(T), HPXHIP_D2D, t.stream()), "sort copy-back");
}
#endif  // HPX_HAVE_HIP_DEVICE_CLOSURES

}  // namespace dev
}}}}  // namespace hpx::parallel::v1::detail
