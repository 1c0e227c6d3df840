// hpx/parallel/algorithms.hpp -- HPX 1.4.0's parallel algorithms over
// hpx::compute::vector iterators, executed by the MI355X kernels behind
// <hpxhip.h>.  Overload sets and result types follow the reference:
//
//   for_each / for_each_n        for_each.hpp:343-423        -> FwdIter
//   fill / fill_n                fill.hpp:158, 261            -> void / FwdIter
//   copy / copy_n                copy.hpp:208, 329            -> tagged_pair<in, out>
//   copy_if                      copy.hpp:584                 -> tagged_pair<in, out>
//   transform (unary)            transform.hpp:303            -> tagged_pair<in, out>
//   transform (binary, 3 / 4 it) transform.hpp:472-506, 624   -> tagged_tuple<in1, in2, out>
//   reduce                       reduce.hpp:200, 271, 344     -> T
//   transform_reduce             transform_reduce.hpp:254     -> T
//   transform_reduce (binary)    transform_reduce_binary.hpp:323, 432 -> T
//   inclusive_scan               inclusive_scan.hpp:288-606   -> FwdIter2
//   exclusive_scan               exclusive_scan.hpp:292, 374  -> FwdIter2
//   transform_inclusive_scan     transform_inclusive_scan.hpp:320, 445
//   transform_exclusive_scan     transform_exclusive_scan.hpp:317
//   sort                         sort.hpp:364                 -> RandomIt
//   sort_by_key                  sort_by_key.hpp:125          -> tagged_pair<keys, values>
//
// Synchronous policies (seq, par, par_unseq) return the value after the
// target's stream is synchronised (the reference's bulk_sync_execute,
// default_executor.hpp:154-195); task policies return hpx::future<...>
// completed by a stream callback (cuda_target.cpp:97-142).
//
// The algorithms run on the executor's target when the policy has one
// (`par.on(exec)`), otherwise on the target of the input iterator; the data
// is always device-resident (compute::vector).  Function objects are mapped
// to device operations by <hpx/compute/hip/functional.hpp>.
#pragma once

#include <hpx/compute/hip.hpp>
#include <hpx/compute/hip/concurrent_executor.hpp>
#include <hpx/compute/hip/default_executor.hpp>
#include <hpx/compute/hip/functional.hpp>
#include <hpx/parallel/detail/device_algorithms.hpp>
#include <hpx/parallel/detail/device_closures.hpp>
#include <hpx/parallel/execution.hpp>
#include <hpx/parallel/segmented_fwd.hpp>

#include <algorithm>
#include <array>
#include <cstring>
#include <functional>
#include <iterator>
#include <tuple>
#include <type_traits>
#include <vector>

namespace hpx { namespace parallel {
inline namespace v1 {

namespace detail {
namespace hip = hpx::compute::hip;
namespace tr = hpx::compute::hip::traits;
using hip::detail::check;

template <typename It>
constexpr bool is_dev = hip::is_device_iterator<typename std::decay<It>::type>::value;
template <typename It>
constexpr bool is_seg = hpx::is_segmented_iterator<typename std::decay<It>::type>::value;
template <typename It>
using value_t = typename std::iterator_traits<It>::value_type;
template <typename T>
constexpr int dt = hip::dtype_of<T>::value;

template <typename P>
using policy_t = typename std::decay<P>::type;
template <typename P>
constexpr bool is_task = policy_t<P>::is_task;

// The target an algorithm runs on, as a non-owning view (same stream; no
// copy, which would get a stream of its own).
template <typename P, typename It>
hip::target target_of(P const& p, It const& it) {
    if constexpr (policy_t<P>::has_executor) {
        return hip::target::view(p.executor().target());
    } else {
        static_assert(is_dev<It>, "raw device pointers need a policy with a HIP executor (par.on(exec))");
        return it.target();
    }
}

template <typename F>
constexpr bool is_complete_binary = tr::detail::is_complete<tr::binary_t<F>>::value;
template <typename F>
constexpr bool is_complete_pred = tr::detail::is_complete<tr::pred_t<F>>::value;
template <typename F>
constexpr bool is_complete_compare = tr::detail::is_complete<tr::compare_t<F>>::value;
// A scan's operator argument: a mapped operator, or any callable op(V, V)
// (an init value is not callable), inclusive_scan.hpp:288 vs :320.
template <typename A, typename V>
constexpr bool is_scan_op = tr::is_binop<A> || std::is_invocable<std::decay_t<A> const&, V const&, V const&>::value;

// Function objects with no mapping to a library operator kind run on kernels
// instantiated for them (device_algorithms.hpp) -- only in a translation
// unit compiled by hipcc.
template <typename F>
void no_device_mapping(char const*) {
    static_assert(compute::hip::detail::dependent_false<F>,
                  "this function object has no mapping to a library operator (traits::unary/binop/pred/compare) "
                  "-- compile the translation unit with hipcc to run it as a device closure");
}

template <typename P>
constexpr bool is_concurrent =
    std::is_same<typename policy_t<P>::executor_type, hip::concurrent_executor>::value;

template <typename It>
auto raw_ptr(It it) {
    if constexpr (std::is_pointer<It>::value) return it;
    else return it.device_ptr();
}

template <typename P, typename R>
using result_t = typename util::detail::algorithm_result<P, R>::type;

// Error contract of every algorithm (dispatch.hpp:122-124, 164-168;
// parallel/exception_list.hpp:20-165): a failure other than std::bad_alloc
// reaches the caller as hpx::exception_list -- thrown under a synchronous
// policy, stored in the returned future under a task policy (including
// failures that surface only when the device work completes: the future is
// flagged so that get() applies the same rule) -- and par_unseq terminates.
template <typename P>
constexpr bool is_unseq = std::is_same<policy_t<P>, execution::parallel_unsequenced_policy>::value;

template <typename P, typename Res, typename Body>
Res guarded(Body&& body) {
    if constexpr (is_unseq<P>) {
        try {
            return body();
        } catch (...) {
            std::terminate();
        }
    } else if constexpr (is_task<P>) {
        try {
            Res f = body();
            if (f.valid()) f.shared()->algorithm_result = true;
            return f;
        } catch (...) {
            return hpx::make_exceptional_future<typename Res::result_type>(
                hpx::detail::to_algorithm_error(std::current_exception()));
        }
    } else {
        try {
            return body();
        } catch (...) {
            std::rethrow_exception(hpx::detail::to_algorithm_error(std::current_exception()));
        }
    }
}

// Finish an algorithm whose device work is queued on t's stream.
template <typename R, typename P, typename Fn>
result_t<P, R> finish(P const&, hip::target const& t, Fn&& fn) {
    if constexpr (is_task<P>) {
        return t.template async_result<R>(
            [fn = std::forward<Fn>(fn)](unsigned char const*) mutable -> R { return fn(); });
    } else {
        t.synchronize();
        if constexpr (std::is_void<R>::value) fn();
        else return fn();
    }
}

// Finish an algorithm whose result (<= 64 bytes) is queued as `kernel ->
// D2H copy into slot.host()`.  value(bytes) forms the result; on_ready(bytes)
// (optional) runs as soon as the bytes are there -- for a task policy on the
// completion callback, before the future becomes ready.  The slot is owned by
// the completion, never by the target (whose stream may belong to a
// temporary policy).
struct no_on_ready {
    void operator()(unsigned char const*) const {}
};
template <typename R, typename P, typename Value, typename OnReady = no_on_ready>
result_t<P, R> finish_slot(P const&, hip::target const& t, hip::result_slot slot, Value value,
                           OnReady on_ready = OnReady()) {
    if constexpr (is_task<P>) {
        return t.template async_result<R>(std::function<R(unsigned char const*)>(std::move(value)), std::move(slot),
                                          std::function<void(unsigned char const*)>(std::move(on_ready)));
    } else {
        t.synchronize();
        auto const* bytes = static_cast<unsigned char const*>(slot.host());
        on_ready(bytes);
        if constexpr (std::is_void<R>::value) value(bytes);
        else return value(bytes);
    }
}

// An elementwise algorithm over n items: launch(target, offset, count) queues
// the kernel(s) for items [offset, offset + count).  With a concurrent_executor
// the range is cut into one chunk per stream (concurrent_executor_parameters:
// chunk = ceil(n / streams)) and the result is ready when every stream is;
// otherwise one launch on the policy's (or the iterator's) target.
template <typename R, typename P, typename It, typename Launch, typename Fn>
result_t<P, R> run_elementwise(P const& p, It const& it, uint64_t n, Launch&& launch, Fn&& fn) {
    if constexpr (is_concurrent<P>) {
        auto const& ex = p.executor().executors();
        uint64_t k = ex.size();
        uint64_t chunk = (n + k - 1) / k;
        std::size_t used = 0;
        for (uint64_t off = 0; off < n; off += chunk, ++used)
            launch(ex[used].target(), off, std::min<uint64_t>(chunk, n - off));
        if constexpr (is_task<P>) {
            std::vector<hpx::future<void>> fs;
            for (std::size_t i = 0; i < std::max<std::size_t>(used, 1); ++i) fs.push_back(ex[i].target().get_future());
            return hpx::when_all(std::move(fs)).then(
                [fn = std::forward<Fn>(fn)](hpx::future<std::vector<hpx::future<void>>>& all) mutable -> R {
                    for (auto& f : all.get()) f.get();
                    return fn();
                });
        } else {
            for (std::size_t i = 0; i < used; ++i) ex[i].target().synchronize();
            if constexpr (std::is_void<R>::value) fn();
            else return fn();
        }
    } else {
        auto const& t = target_of(p, it);
        launch(t, uint64_t(0), n);
        return finish<R>(p, t, std::forward<Fn>(fn));
    }
}

// Queue the D2H copy of a result slot's first `bytes` bytes.
inline void fetch_slot(hip::target const& t, hip::result_slot const& slot, std::size_t bytes, char const* what) {
    check(hpxhip_memcpy_async(const_cast<void*>(slot.host()), slot.device(), bytes, HPXHIP_D2H, t.stream()), what);
}

template <typename T>
struct load_value {
    T operator()(unsigned char const* b) const {
        T v;
        std::memcpy(&v, b, sizeof(T));
        return v;
    }
};

template <typename It>
uint64_t distance(It first, It last) {
    auto d = last - first;
    if (d < 0) throw hpx::exception(HPXHIP_ERROR_INVALID_ARGUMENT, "negative range");
    return static_cast<uint64_t>(d);
}

// Pointer behind a contiguous host iterator (std::vector<T>::iterator / T*).
template <typename It>
auto host_ptr(It it) {
    return &*it;
}

}  // namespace detail
namespace algo {

// ------------------------------------------------------------- for_each
// A function object with a traits::unary mapping runs on the library kernel;
// any other callable runs on a kernel instantiated for it when the TU is
// compiled by hipcc (detail/device_closures.hpp), else it does not compile.
template <typename P, typename It, typename F>
detail::result_t<P, It> for_each(P&& p, It first, It last, F&& f) {
    if constexpr (detail::is_seg<It>) {
        return segmented_detail::for_each(std::forward<P>(p), first, last, std::forward<F>(f));
    } else {
    static_assert(detail::is_dev<It>, "for_each: device iterators required");
    using T = detail::value_t<It>;
    uint64_t n = detail::distance(first, last);
    T* base = first.device_ptr();
    return detail::run_elementwise<It>(
        p, first, n,
        [&](auto const& t, uint64_t off, uint64_t cnt) {
            if constexpr (detail::tr::is_unary<F>) {
                using Tr = detail::tr::unary_t<F>;
                T s[2] = {};
                Tr::scalars(f, s);
                detail::check(hpxhip_for_each(detail::dt<T>, Tr::kind, s, base + off, cnt, t.stream()), "for_each");
            } else {
                detail::device_for_each(t, f, base + off, cnt);
            }
        },
        [last] { return last; });
    }
}

template <typename P, typename It, typename Size, typename F>
detail::result_t<P, It> for_each_n(P&& p, It first, Size count, F&& f) {
    if (count <= 0) {
        if constexpr (detail::is_task<P>) return hpx::make_ready_future(first);
        else return first;
    }
    return for_each(std::forward<P>(p), first, first + count, std::forward<F>(f));
}

// ------------------------------------------------------------------ fill
template <typename P, typename It, typename T>
detail::result_t<P, void> fill(P&& p, It first, It last, T value) {
    if constexpr (detail::is_seg<It>) {
        return segmented_detail::fill(std::forward<P>(p), first, last, value);
    } else {
    static_assert(detail::is_dev<It>, "fill: device iterators required");
    using V = detail::value_t<It>;
    V v = static_cast<V>(value);
    V* base = first.device_ptr();
    return detail::run_elementwise<void>(
        p, first, detail::distance(first, last),
        [&](auto const& t, uint64_t off, uint64_t cnt) {
            detail::check(hpxhip_fill(detail::dt<V>, &v, base + off, cnt, t.stream()), "fill");
        },
        [] {});
    }
}

template <typename P, typename It, typename Size, typename T>
detail::result_t<P, It> fill_n(P&& p, It first, Size count, T value) {
    static_assert(detail::is_dev<It>, "fill_n: device iterators required");
    using V = detail::value_t<It>;
    uint64_t n = count > 0 ? static_cast<uint64_t>(count) : 0;
    V v = static_cast<V>(value);
    V* base = first.device_ptr();
    It end = first + static_cast<std::ptrdiff_t>(n);
    return detail::run_elementwise<It>(
        p, first, n,
        [&](auto const& t, uint64_t off, uint64_t cnt) {
            detail::check(hpxhip_fill(detail::dt<V>, &v, base + off, cnt, t.stream()), "fill_n");
        },
        [end] { return end; });
}

// ------------------------------------------------------------------ copy
template <typename P, typename In, typename Out>
detail::result_t<P, util::tagged_pair<In, Out>> copy(P&& p, In first, In last, Out dest) {
    using R = util::tagged_pair<In, Out>;
    if constexpr (detail::is_seg<In> || detail::is_seg<Out>) {
        return segmented_detail::copy(std::forward<P>(p), first, last, dest);
    } else {
    uint64_t n = detail::distance(first, last);
    if constexpr (detail::is_dev<In> && detail::is_dev<Out>) {
        using T = detail::value_t<In>;
        static_assert(std::is_same<T, detail::value_t<Out>>::value, "copy: element types must match");
        T const* in = first.device_ptr();
        T* out = dest.device_ptr();
        Out end = dest + static_cast<std::ptrdiff_t>(n);
        return detail::run_elementwise<R>(
            p, first, n,
            [&](auto const& t, uint64_t off, uint64_t cnt) {
                detail::check(hpxhip_copy(detail::dt<T>, in + off, out + off, cnt, t.stream()), "copy");
            },
            [last, end] { return R{last, end}; });
    } else if constexpr (detail::is_dev<In>) {  // device -> host
        using T = detail::value_t<In>;
        auto const& t = detail::target_of(p, first);
        if (n)
            detail::check(hpxhip_memcpy_async(detail::host_ptr(dest), first.device_ptr(), n * sizeof(T), HPXHIP_D2H,
                                              t.stream()),
                          "copy (D2H)");
        Out end = dest + static_cast<std::ptrdiff_t>(n);
        return detail::finish<R>(p, t, [last, end] { return R{last, end}; });
    } else {  // host -> device
        static_assert(detail::is_dev<Out>, "copy: at least one side must be a device iterator");
        using T = detail::value_t<Out>;
        auto const& t = detail::target_of(p, dest);
        if (n)
            detail::check(hpxhip_memcpy_async(dest.device_ptr(), detail::host_ptr(first), n * sizeof(T), HPXHIP_H2D,
                                              t.stream()),
                          "copy (H2D)");
        Out end = dest + static_cast<std::ptrdiff_t>(n);
        return detail::finish<R>(p, t, [last, end] { return R{last, end}; });
    }
    }
}

template <typename P, typename In, typename Size, typename Out>
detail::result_t<P, util::tagged_pair<In, Out>> copy_n(P&& p, In first, Size count, Out dest) {
    std::ptrdiff_t n = count > 0 ? static_cast<std::ptrdiff_t>(count) : 0;
    return copy(std::forward<P>(p), first, first + n, dest);
}

// --------------------------------------------------------------- copy_if
template <typename P, typename In, typename Out, typename F>
detail::result_t<P, util::tagged_pair<In, Out>> copy_if(P&& p, In first, In last, Out dest, F&& f) {
    static_assert(detail::is_dev<In> && detail::is_dev<Out>, "copy_if: device iterators required");
    using T = detail::value_t<In>;
    using R = util::tagged_pair<In, Out>;
    auto const& t = detail::target_of(p, first);
    uint64_t n = detail::distance(first, last);
    auto slot = t.make_result_slot();
    if constexpr (detail::is_complete_pred<F>) {
        using Tr = detail::tr::pred_t<F>;
        T arg = static_cast<T>(Tr::arg(f));
        detail::check(hpxhip_copy_if(detail::dt<T>, Tr::kind, &arg, first.device_ptr(), dest.device_ptr(), n,
                                     static_cast<uint64_t*>(slot.device()), t.stream(), nullptr, 0),
                      "copy_if");
    } else {
#if HPX_HAVE_HIP_DEVICE_CLOSURES
        detail::dev::copy_if(t, static_cast<T const*>(first.device_ptr()), dest.device_ptr(), n, f,
                             static_cast<uint64_t*>(slot.device()));
#else
        detail::no_device_mapping<F>("copy_if");
#endif
    }
    detail::fetch_slot(t, slot, 8, "copy_if count");
    return detail::finish_slot<R>(p, t, std::move(slot), [last, dest](unsigned char const* b) {
        uint64_t c;
        std::memcpy(&c, b, 8);
        return R{last, dest + static_cast<std::ptrdiff_t>(c)};
    });
}

// ------------------------------------------------------------- transform
template <typename P, typename In, typename Out, typename F>
detail::result_t<P, util::tagged_pair<In, Out>> transform(P&& p, In first, In last, Out dest, F&& f) {
    if constexpr (detail::is_seg<In>) {
        return segmented_detail::transform(std::forward<P>(p), first, last, dest, std::forward<F>(f));
    } else {
    static_assert(detail::is_dev<In> && detail::is_dev<Out>, "transform: device iterators required");
    using TI = detail::value_t<In>;
    using TO = detail::value_t<Out>;
    using R = util::tagged_pair<In, Out>;
    uint64_t n = detail::distance(first, last);
    TI const* in = first.device_ptr();
    TO* out = dest.device_ptr();
    Out end = dest + static_cast<std::ptrdiff_t>(n);
    return detail::run_elementwise<R>(
        p, first, n,
        [&](auto const& t, uint64_t off, uint64_t cnt) {
            if constexpr (detail::tr::is_unary<F>) {
                using Tr = detail::tr::unary_t<F>;
                using C = detail::tr::compute_t<Tr, F, TI>;
                C s[2] = {};
                Tr::scalars(f, s);
                detail::check(hpxhip_transform(detail::dt<TI>, detail::dt<C>, detail::dt<TO>, Tr::kind, s, in + off,
                                               out + off, cnt, t.stream()),
                              "transform");
            } else {
                detail::device_transform(t, f, in + off, out + off, cnt);
            }
        },
        [last, end] { return R{last, end}; });
    }
}

}  // namespace algo
namespace detail {
template <typename P, typename In1, typename In2, typename Out, typename F>
result_t<P, util::tagged_tuple<In1, In2, Out>> transform_binary(P&& p, In1 first1, uint64_t n, In2 first2, Out dest,
                                                                F&& f) {
    if constexpr (is_seg<In1>) {
        return segmented_detail::transform_binary(std::forward<P>(p), first1, n, first2, dest, std::forward<F>(f));
    } else {
    static_assert(is_dev<In1> && is_dev<In2> && is_dev<Out>, "transform: device iterators required");
    using T = value_t<In1>;
    using T2 = value_t<In2>;
    using TO = value_t<Out>;
    using R = util::tagged_tuple<In1, In2, Out>;
    T const* a = first1.device_ptr();
    T2 const* b = first2.device_ptr();
    TO* out = dest.device_ptr();
    auto d = static_cast<std::ptrdiff_t>(n);
    In1 e1 = first1 + d;
    In2 e2 = first2 + d;
    Out eo = dest + d;
    return run_elementwise<R>(
        p, first1, n,
        [&](auto const& t, uint64_t off, uint64_t cnt) {
            if constexpr (is_complete_binary<F>) {
                static_assert(std::is_same<T, T2>::value, "transform: input element types must match");
                using Tr = tr::binary_t<F>;
                using C = tr::compute_t<Tr, F, T>;
                C s[2] = {};
                Tr::scalars(f, s);
                check(hpxhip_transform_binary(dt<T>, dt<C>, dt<TO>, Tr::kind, s, a + off, b + off, out + off, cnt,
                                              t.stream()),
                      "transform");
            } else {
                device_transform2(t, f, a + off, b + off, out + off, cnt);
            }
        },
        [e1, e2, eo] { return R{e1, e2, eo}; });
    }
}
}  // namespace detail
namespace algo {

template <typename P, typename In1, typename In2, typename Out, typename F,
          typename = typename std::enable_if<detail::is_dev<Out> || detail::is_seg<Out>>::type>
detail::result_t<P, util::tagged_tuple<In1, In2, Out>> transform(P&& p, In1 first1, In1 last1, In2 first2, Out dest,
                                                                F&& f) {
    return detail::transform_binary(std::forward<P>(p), first1, detail::distance(first1, last1), first2, dest,
                                    std::forward<F>(f));
}

template <typename P, typename In1, typename In2, typename Out, typename F>
detail::result_t<P, util::tagged_tuple<In1, In2, Out>> transform(P&& p, In1 first1, In1 last1, In2 first2, In2 last2,
                                                                Out dest, F&& f) {
    uint64_t n = std::min(detail::distance(first1, last1), detail::distance(first2, last2));
    return detail::transform_binary(std::forward<P>(p), first1, n, first2, dest, std::forward<F>(f));
}

// ------------------------------------------------------------ reductions
}  // namespace algo
namespace detail {
// *out_dev <- init (op) conv(x_0) (op) ... over [first, first + n), queued on
// t's stream (the library kernel for mapped functors, a kernel instantiated
// for a device closure otherwise).
template <typename T, typename TI, typename Op, typename Conv>
void reduce_into(hip::target const& t, TI const* first, uint64_t n, T init, Op const& op, Conv const& conv,
                 void* out_dev) {
    if constexpr (tr::is_binop<Op> && tr::is_unary<Conv>) {
        T s[2] = {};
        tr::unary_t<Conv>::scalars(conv, s);
        check(hpxhip_transform_reduce(dt<TI>, dt<T>, tr::binop_t<Op>::kind, tr::unary_t<Conv>::kind, s, &init, first, n,
                                      out_dev, t.stream(), nullptr, 0),
              "transform_reduce");
    } else {
#if HPX_HAVE_HIP_DEVICE_CLOSURES
        dev::reduce<T, false>(t, first, static_cast<TI const*>(nullptr), n, init, op, conv, out_dev);
#else
        no_device_mapping<Op>("transform_reduce");
#endif
    }
}

// [first, first + n) scanned into out, queued on t's stream; prefix_dev (a
// device value, built-in operators only) replaces init when given.
template <typename V, typename Op, typename Conv, typename T>
void scan_into(hip::target const& t, V const* first, V* out, uint64_t n, Op const& op, Conv const& conv, T init,
               V const* prefix_dev, bool inclusive) {
    if constexpr (tr::is_binop<Op> && tr::is_unary<Conv>) {
        V s[2] = {};
        tr::unary_t<Conv>::scalars(conv, s);
        V iv = static_cast<V>(init);
        check(hpxhip_scan(dt<V>, tr::binop_t<Op>::kind, inclusive ? 1 : 0, tr::unary_t<Conv>::kind, s, &iv, prefix_dev,
                          first, out, n, t.stream(), nullptr, 0),
              inclusive ? "inclusive_scan" : "exclusive_scan");
    } else {
#if HPX_HAVE_HIP_DEVICE_CLOSURES
        if (prefix_dev)
            throw hpx::exception(HPXHIP_ERROR_UNSUPPORTED, "scan: a device prefix needs a built-in operator");
        dev::scan(t, first, out, n, op, conv, init, inclusive);
#else
        no_device_mapping<Op>(inclusive ? "inclusive_scan" : "exclusive_scan");
#endif
    }
}

template <typename T, typename P, typename It, typename Op, typename Conv>
result_t<P, T> reduce_impl(P&& p, It first, It last, T init, Op&& op, Conv&& conv) {
    if constexpr (is_seg<It>) {
        return segmented_detail::reduce<T>(std::forward<P>(p), first, last, init, std::forward<Op>(op),
                                           std::forward<Conv>(conv));
    } else {
    static_assert(is_dev<It>, "reduce: device iterators required");
    using TI = value_t<It>;
    auto const& t = target_of(p, first);
    auto slot = t.make_result_slot();
    reduce_into<T>(t, static_cast<TI const*>(first.device_ptr()), distance(first, last), init, op, conv, slot.device());
    fetch_slot(t, slot, sizeof(T), "reduce result");
    return finish_slot<T>(p, t, std::move(slot), load_value<T>{});
    }
}
}  // namespace detail
namespace algo {

template <typename P, typename It, typename T, typename Op>
detail::result_t<P, T> reduce(P&& p, It first, It last, T init, Op&& op) {
    return detail::reduce_impl<T>(std::forward<P>(p), first, last, init, std::forward<Op>(op),
                                  hpx::compute::hip::functional::identity{});
}
template <typename P, typename It, typename T>
detail::result_t<P, T> reduce(P&& p, It first, It last, T init) {
    return reduce(std::forward<P>(p), first, last, init, std::plus<T>());
}
template <typename P, typename It>
detail::result_t<P, detail::value_t<It>> reduce(P&& p, It first, It last) {
    using T = detail::value_t<It>;
    return reduce(std::forward<P>(p), first, last, T(), std::plus<T>());
}

template <typename P, typename It, typename T, typename Red, typename Conv,
          typename = typename std::enable_if<detail::is_dev<It> || detail::is_seg<It>>::type>
detail::result_t<P, T> transform_reduce(P&& p, It first, It last, T init, Red&& red, Conv&& conv) {
    return detail::reduce_impl<T>(std::forward<P>(p), first, last, init, std::forward<Red>(red),
                                  std::forward<Conv>(conv));
}

}  // namespace algo
namespace detail {
template <typename T, typename P, typename It1, typename It2, typename Red, typename Comb>
result_t<P, T> reduce_binary_impl(P&& p, It1 first1, It1 last1, It2 first2, T init, Red&& red, Comb&& comb) {
    static_assert(is_dev<It1> && is_dev<It2>, "transform_reduce: device iterators required");
    using TI = value_t<It1>;
    static_assert(std::is_same<TI, value_t<It2>>::value, "transform_reduce: input element types must match");
    auto const& t = target_of(p, first1);
    auto slot = t.make_result_slot();
    if constexpr (tr::is_binop<Red> && is_complete_binary<Comb>) {
        T s[2] = {};
        tr::binary_t<Comb>::scalars(comb, s);
        check(hpxhip_transform_reduce_binary(dt<TI>, dt<T>, tr::binop_t<Red>::kind, tr::binary_t<Comb>::kind, s,
                                             &init, first1.device_ptr(), first2.device_ptr(), distance(first1, last1),
                                             slot.device(), t.stream(), nullptr, 0),
              "transform_reduce");
    } else {
#if HPX_HAVE_HIP_DEVICE_CLOSURES
        dev::reduce<T, true>(t, static_cast<TI const*>(first1.device_ptr()), static_cast<TI const*>(first2.device_ptr()),
                             distance(first1, last1), init, red, comb, slot.device());
#else
        no_device_mapping<Comb>("transform_reduce");
#endif
    }
    fetch_slot(t, slot, sizeof(T), "reduce result");
    return finish_slot<T>(p, t, std::move(slot), load_value<T>{});
}
}  // namespace detail
namespace algo {

// transform_reduce_binary.hpp:323 -- inner product with std::plus / std::multiplies
template <typename P, typename It1, typename It2, typename T,
          typename = typename std::enable_if<detail::is_dev<It2>>::type>
detail::result_t<P, T> transform_reduce(P&& p, It1 first1, It1 last1, It2 first2, T init) {
    return detail::reduce_binary_impl<T>(std::forward<P>(p), first1, last1, first2, init, std::plus<T>(),
                                         std::multiplies<T>());
}
// transform_reduce_binary.hpp:432
template <typename P, typename It1, typename It2, typename T, typename Red, typename Comb,
          typename = typename std::enable_if<detail::is_dev<It2>>::type>
detail::result_t<P, T> transform_reduce(P&& p, It1 first1, It1 last1, It2 first2, T init, Red&& red, Comb&& comb) {
    return detail::reduce_binary_impl<T>(std::forward<P>(p), first1, last1, first2, init, std::forward<Red>(red),
                                         std::forward<Comb>(comb));
}

// ------------------------------------------------------------------ scans
}  // namespace algo
namespace detail {
template <typename P, typename In, typename Out, typename Op, typename Conv, typename T>
result_t<P, Out> scan_impl(P&& p, In first, In last, Out dest, Op&& op, Conv&& conv, T init, bool inclusive) {
    if constexpr (is_seg<In>) {
        return segmented_detail::scan(std::forward<P>(p), first, last, dest, std::forward<Op>(op),
                                      std::forward<Conv>(conv), init, inclusive);
    } else {
    static_assert(is_dev<In> && is_dev<Out>, "scan: device iterators required");
    using V = value_t<In>;
    static_assert(std::is_same<V, value_t<Out>>::value, "scan: input and output element types must match");
    auto const& t = target_of(p, first);
    uint64_t n = distance(first, last);
    scan_into(t, static_cast<V const*>(first.device_ptr()), dest.device_ptr(), n, op, conv, init,
              static_cast<V const*>(nullptr), inclusive);
    Out end = dest + static_cast<std::ptrdiff_t>(n);
    return finish<Out>(p, t, [end] { return end; });
    }
}
using ident = hpx::compute::hip::functional::identity;
}  // namespace detail
namespace algo {

// inclusive_scan.hpp:288 (op, init) and :320 (init, op)
template <typename P, typename In, typename Out, typename A, typename B>
detail::result_t<P, Out> inclusive_scan(P&& p, In first, In last, Out dest, A&& a, B&& b) {
    if constexpr (detail::is_scan_op<A, detail::value_t<In>>)
        return detail::scan_impl(std::forward<P>(p), first, last, dest, std::forward<A>(a), detail::ident{}, b, true);
    else
        return detail::scan_impl(std::forward<P>(p), first, last, dest, std::forward<B>(b), detail::ident{}, a, true);
}
// inclusive_scan.hpp:409 (init) and :511 (op; init = value_type())
template <typename P, typename In, typename Out, typename A>
detail::result_t<P, Out> inclusive_scan(P&& p, In first, In last, Out dest, A&& a) {
    using V = detail::value_t<In>;
    if constexpr (detail::is_scan_op<A, V>)
        return detail::scan_impl(std::forward<P>(p), first, last, dest, std::forward<A>(a), detail::ident{}, V(), true);
    else
        return detail::scan_impl(std::forward<P>(p), first, last, dest, std::plus<V>(), detail::ident{}, a, true);
}
// inclusive_scan.hpp:591
template <typename P, typename In, typename Out>
detail::result_t<P, Out> inclusive_scan(P&& p, In first, In last, Out dest) {
    using V = detail::value_t<In>;
    return detail::scan_impl(std::forward<P>(p), first, last, dest, std::plus<V>(), detail::ident{}, V(), true);
}

// exclusive_scan.hpp:292 (init, op) and :374 (init)
template <typename P, typename In, typename Out, typename T, typename Op>
detail::result_t<P, Out> exclusive_scan(P&& p, In first, In last, Out dest, T init, Op&& op) {
    return detail::scan_impl(std::forward<P>(p), first, last, dest, std::forward<Op>(op), detail::ident{}, init, false);
}
template <typename P, typename In, typename Out, typename T>
detail::result_t<P, Out> exclusive_scan(P&& p, In first, In last, Out dest, T init) {
    using V = detail::value_t<In>;
    return detail::scan_impl(std::forward<P>(p), first, last, dest, std::plus<V>(), detail::ident{}, init, false);
}

// transform_inclusive_scan.hpp:320 (op, conv, init) and :445 (op, conv)
template <typename P, typename In, typename Out, typename Op, typename Conv, typename T>
detail::result_t<P, Out> transform_inclusive_scan(P&& p, In first, In last, Out dest, Op&& op, Conv&& conv, T init) {
    return detail::scan_impl(std::forward<P>(p), first, last, dest, std::forward<Op>(op), std::forward<Conv>(conv),
                             init, true);
}
template <typename P, typename In, typename Out, typename Op, typename Conv>
detail::result_t<P, Out> transform_inclusive_scan(P&& p, In first, In last, Out dest, Op&& op, Conv&& conv) {
    using V = detail::value_t<In>;
    return detail::scan_impl(std::forward<P>(p), first, last, dest, std::forward<Op>(op), std::forward<Conv>(conv),
                             V(), true);
}
// transform_exclusive_scan.hpp:317 (init, op, conv)
template <typename P, typename In, typename Out, typename T, typename Op, typename Conv>
detail::result_t<P, Out> transform_exclusive_scan(P&& p, In first, In last, Out dest, T init, Op&& op, Conv&& conv) {
    return detail::scan_impl(std::forward<P>(p), first, last, dest, std::forward<Op>(op), std::forward<Conv>(conv),
                             init, false);
}

// ------------------------------------------------------------------- sort
// sort.hpp:364 sort(policy, first, last, comp = less, proj = identity):
// std::less / std::greater on the elements themselves take the radix sort
// (hpxhip_sort); any other comparator or projection a comparison merge sort
// instantiated for it (hipcc translation units, device_algorithms.hpp).
template <typename P, typename It, typename Comp = std::less<>, typename Proj = util::projection_identity,
          typename = std::enable_if_t<detail::is_dev<It>>>
detail::result_t<P, It> sort(P&& p, It first, It last, Comp&& comp = Comp(), Proj&& proj = Proj()) {
    using T = detail::value_t<It>;
    auto const& t = detail::target_of(p, first);
    uint64_t n = detail::distance(first, last);
    if constexpr (detail::is_complete_compare<Comp> &&
                  std::is_same<std::decay_t<Proj>, util::projection_identity>::value) {
        detail::check(hpxhip_sort(detail::dt<T>, first.device_ptr(), n,
                                  detail::tr::compare_t<Comp>::descending ? 1 : 0, t.stream(), nullptr, 0),
                      "sort");
    } else {
#if HPX_HAVE_HIP_DEVICE_CLOSURES
        detail::dev::merge_sort(t, first.device_ptr(), n, comp, proj);
#else
        detail::no_device_mapping<Comp>("sort");
#endif
    }
    return detail::finish<It>(p, t, [last] { return last; });
}

// container_algorithms/sort.hpp:102: sort(policy, rng[, comp[, proj]]) over
// begin(rng), end(rng).
template <typename P, typename Rng, typename Comp = std::less<>, typename Proj = util::projection_identity,
          typename = std::enable_if_t<detail::is_dev<decltype(std::declval<Rng&>().begin())>>>
auto sort(P&& p, Rng&& rng, Comp&& comp = Comp(), Proj&& proj = Proj()) {
    return sort(std::forward<P>(p), rng.begin(), rng.end(), std::forward<Comp>(comp), std::forward<Proj>(proj));
}

// is_sorted.hpp:40-120: no adjacent pair ordered after one another under
// comp (std::less / std::greater), counted on the device.
template <typename P, typename It, typename Comp = std::less<>>
detail::result_t<P, bool> is_sorted(P&& p, It first, It last, Comp&& = Comp()) {
    static_assert(detail::is_dev<It>, "is_sorted: device iterators required");
    using T = detail::value_t<It>;
    auto const& t = detail::target_of(p, first);
    auto slot = t.make_result_slot();
    detail::check(hpxhip_unsorted_pairs(detail::dt<T>, first.device_ptr(), detail::distance(first, last),
                                        detail::tr::compare_t<Comp>::descending ? 1 : 0,
                                        static_cast<uint64_t*>(slot.device()), t.stream()),
                  "is_sorted");
    detail::fetch_slot(t, slot, 8, "is_sorted count");
    return detail::finish_slot<bool>(p, t, std::move(slot), [](unsigned char const* b) {
        uint64_t c;
        std::memcpy(&c, b, 8);
        return c == 0;
    });
}

template <typename P, typename KeyIt, typename ValIt, typename Comp = std::less<>>
detail::result_t<P, util::tagged_pair<KeyIt, ValIt>> sort_by_key(P&& p, KeyIt key_first, KeyIt key_last,
                                                                 ValIt value_first, Comp&& = Comp()) {
    static_assert(detail::is_dev<KeyIt> && detail::is_dev<ValIt>, "sort_by_key: device iterators required");
    using K = detail::value_t<KeyIt>;
    using V = detail::value_t<ValIt>;
    using R = util::tagged_pair<KeyIt, ValIt>;
    auto const& t = detail::target_of(p, key_first);
    uint64_t n = detail::distance(key_first, key_last);
    detail::check(hpxhip_sort_by_key(detail::dt<K>, detail::dt<V>, key_first.device_ptr(), value_first.device_ptr(),
                                     n, detail::tr::compare_t<Comp>::descending ? 1 : 0, t.stream(), nullptr, 0),
                  "sort_by_key");
    ValIt vend = value_first + static_cast<std::ptrdiff_t>(n);
    return detail::finish<R>(p, t, [key_last, vend] { return R{key_last, vend}; });
}

// ------------------------------------------------------------------ merge
// merge.hpp:476: stable (first range first on ties), ascending / descending.
template <typename P, typename In1, typename In2, typename Out, typename Comp = std::less<>>
detail::result_t<P, util::tagged_tuple<In1, In2, Out>> merge(P&& p, In1 first1, In1 last1, In2 first2, In2 last2,
                                                            Out dest, Comp&& = Comp()) {
    static_assert(detail::is_dev<In1> && detail::is_dev<In2> && detail::is_dev<Out>, "merge: device iterators required");
    using T = detail::value_t<In1>;
    static_assert(std::is_same<T, detail::value_t<In2>>::value && std::is_same<T, detail::value_t<Out>>::value,
                  "merge: one element type");
    using R = util::tagged_tuple<In1, In2, Out>;
    auto const& t = detail::target_of(p, first1);
    uint64_t n1 = detail::distance(first1, last1), n2 = detail::distance(first2, last2);
    detail::check(hpxhip_merge(detail::dt<T>, first1.device_ptr(), n1, first2.device_ptr(), n2, dest.device_ptr(),
                               detail::tr::compare_t<Comp>::descending ? 1 : 0, t.stream(), nullptr, 0),
                  "merge");
    Out end = dest + static_cast<std::ptrdiff_t>(n1 + n2);
    return detail::finish<R>(p, t, [last1, last2, end] { return R{last1, last2, end}; });
}

}  // namespace algo
// --------------------------------------------------------------- for_loop
// for_loop_induction.hpp:210-219: an induction over an iterator, value at
// iteration i = it + stride * i (stride 1 on the device: contiguous kernels).
template <typename It>
struct induction_stride_helper {
    It var_;
    std::size_t stride_;
};
template <typename It>
induction_stride_helper<It> induction(It it, std::size_t stride = 1) {
    return induction_stride_helper<It>{it, stride};
}

// for_loop_reduction.hpp:35-132: reduction(var, identity, combiner).  The
// reference keeps one view per OS thread and folds `var = op(var, view_k)`
// at loop exit (62-66); here one launch forms a single view (the
// transform_reduce kernel with init = identity) and the exit folds it into
// var.  Equal to the reference for a neutral identity (every helper below
// without an explicit identity); with a non-neutral explicit identity the
// reference's result depends on its OS thread count.
template <typename T, typename Op>
struct reduction_helper {
    T& var_;
    T identity_;
    Op op_;
};
template <typename T, typename Op>
reduction_helper<T, typename std::decay<Op>::type> reduction(T& var, T const& identity, Op&& combiner) {
    return {var, identity, std::forward<Op>(combiner)};
}
template <typename T> reduction_helper<T, std::plus<T>> reduction_plus(T& var) { return {var, T(), {}}; }
template <typename T> reduction_helper<T, std::plus<T>> reduction_plus(T& var, T const& id) { return {var, id, {}}; }
template <typename T> reduction_helper<T, std::multiplies<T>> reduction_multiplies(T& var) { return {var, T(1), {}}; }
template <typename T> reduction_helper<T, std::multiplies<T>> reduction_multiplies(T& var, T const& id) {
    return {var, id, {}};
}
template <typename T> reduction_helper<T, std::bit_and<T>> reduction_bit_and(T& var) { return {var, ~T(), {}}; }
template <typename T> reduction_helper<T, std::bit_and<T>> reduction_bit_and(T& var, T const& id) {
    return {var, id, {}};
}
template <typename T> reduction_helper<T, std::bit_or<T>> reduction_bit_or(T& var) { return {var, T(), {}}; }
template <typename T> reduction_helper<T, std::bit_or<T>> reduction_bit_or(T& var, T const& id) { return {var, id, {}}; }
template <typename T> reduction_helper<T, std::bit_xor<T>> reduction_bit_xor(T& var) { return {var, T(), {}}; }
template <typename T> reduction_helper<T, std::bit_xor<T>> reduction_bit_xor(T& var, T const& id) {
    return {var, id, {}};
}
template <typename T> reduction_helper<T, compute::hip::functional::minimum> reduction_min(T& var) {
    return {var, var, {}};
}
template <typename T> reduction_helper<T, compute::hip::functional::minimum> reduction_min(T& var, T const& id) {
    return {var, id, {}};
}
template <typename T> reduction_helper<T, compute::hip::functional::maximum> reduction_max(T& var) {
    return {var, var, {}};
}
template <typename T> reduction_helper<T, compute::hip::functional::maximum> reduction_max(T& var, T const& id) {
    return {var, id, {}};
}

namespace detail {
template <typename It>
It loop_var(It it) { return it; }
template <typename T, typename Op>
reduction_helper<T, Op> const& loop_var(reduction_helper<T, Op> const& r) { return r; }
template <typename It>
It loop_var(induction_stride_helper<It> const& h) { return h.var_; }
// the stride of each loop variable (for_loop_induction.hpp:210-219)
template <typename It>
int64_t loop_stride(It const&) { return 1; }
template <typename It>
int64_t loop_stride(induction_stride_helper<It> const& h) { return static_cast<int64_t>(h.stride_); }
template <typename T, typename Op>
int64_t loop_stride(reduction_helper<T, Op> const&) { return 1; }
template <std::size_t N>
using strides_t = std::array<int64_t, N>;
// One reduction's share of a reduction loop: its body's inputs feed the
// transform_reduce kernels, the view lands at `out` (device) and `fold`
// returns the exit_iteration that folds it into the live-out variable
// (for_loop_reduction.hpp:60-66).
template <typename Vars, std::size_t N, std::size_t Red, typename F, std::size_t... In>
std::function<void(unsigned char const*)> launch_accumulate(
    hip::target const& t, Vars const& v, strides_t<N> const& st, uint64_t n,
    compute::hip::functional::loop_accumulate<Red, F, In...> const& b, void* out) {
    if (((st[In] != 1) || ...))
        throw hpx::exception(HPXHIP_ERROR_UNSUPPORTED,
                             "for_loop_n: a reduction loop reads its inductions with stride 1 (the transform_reduce "
                             "kernels are contiguous)");
    auto const& red = std::get<Red>(v);
    using T = std::decay_t<decltype(red.identity_)>;
    using Op = std::decay_t<decltype(red.op_)>;
    static_assert(std::is_same<std::decay_t<decltype(red)>, reduction_helper<T, Op>>::value,
                  "loop_accumulate: position Red must name one of the loop's reductions");
    static_assert(sizeof(T) <= 8, "for_loop reductions of up to 8-byte types");
    auto ins = std::make_tuple(std::get<In>(v)...);
    auto in0 = std::get<0>(ins);
    using TI = value_t<decltype(in0)>;
    T s[2] = {};
    T init = red.identity_;
    if constexpr (sizeof...(In) == 1) {
        tr::unary_t<F>::scalars(b.f, s);
        check(hpxhip_transform_reduce(dt<TI>, dt<T>, tr::binop_t<Op>::kind, tr::unary_t<F>::kind, s, &init,
                                      raw_ptr(in0), n, out, t.stream(), nullptr, 0),
              "for_loop_n");
    } else {
        auto in1 = std::get<1>(ins);
        static_assert(std::is_same<TI, value_t<decltype(in1)>>::value, "for_loop_n: both inputs need one element type");
        tr::binary_t<F>::scalars(b.f, s);
        check(hpxhip_transform_reduce_binary(dt<TI>, dt<T>, tr::binop_t<Op>::kind, tr::binary_t<F>::kind, s, &init,
                                             raw_ptr(in0), raw_ptr(in1), n, out, t.stream(), nullptr, 0),
              "for_loop_n");
    }
    T* var = &red.var_;
    Op op = red.op_;
    return [var, op](unsigned char const* bytes) {
        T view;
        std::memcpy(&view, bytes, sizeof(T));
        *var = op(*var, view);
    };
}

template <typename T>
struct is_reduction : std::false_type {};
template <typename T, typename Op>
struct is_reduction<reduction_helper<T, Op>> : std::true_type {};
template <typename Vars, std::size_t... I>
constexpr std::size_t count_reductions(std::index_sequence<I...>) {
    return (std::size_t(0) + ... + (is_reduction<std::decay_t<std::tuple_element_t<I, Vars>>>::value ? 1 : 0));
}
template <std::size_t... R>
constexpr bool distinct_positions() {
    constexpr std::size_t r[] = {R...};
    for (std::size_t i = 0; i < sizeof...(R); ++i)
        for (std::size_t j = i + 1; j < sizeof...(R); ++j)
            if (r[i] == r[j]) return false;
    return true;
}

// The reduction loop: every reduction's kernels on the loop's stream, the
// views back in one result slot (8 bytes each), and one exit_iteration that
// folds all of them -- under par(task) on the completion, so the live-out
// variables are final once the future is ready (not only after get()).
template <typename P, typename Vars, std::size_t N, typename... A>
result_t<P, void> for_loop_reductions(P&& p, Vars const& v, strides_t<N> const& st, uint64_t n, A const&... parts) {
    static_assert(distinct_positions<A::red...>(), "for_loop: each reduction is accumulated by one body");
    static_assert(count_reductions<Vars>(std::make_index_sequence<N>{}) == sizeof...(A),
                  "for_loop: every reduction argument needs a loop_accumulate in the body");
    auto const& t = target_of(p, std::get<0>(v));
    auto slot = t.make_result_slot();
    std::vector<std::function<void(unsigned char const*)>> folds;
    std::size_t k = 0;
    (folds.push_back(launch_accumulate(t, v, st, n, parts, static_cast<char*>(slot.device()) + 8 * k++)), ...);
    fetch_slot(t, slot, 8 * sizeof...(A), "for_loop_n result");
    return finish_slot<void>(p, t, std::move(slot), [](unsigned char const*) {},
                             [folds = std::move(folds)](unsigned char const* b) {
                                 for (std::size_t i = 0; i < folds.size(); ++i) folds[i](b + 8 * i);
                             });
}
template <typename P, typename Vars, std::size_t N, std::size_t Red, typename F, std::size_t... In>
result_t<P, void> for_loop_body(P&& p, Vars const& v, strides_t<N> const& st, uint64_t n,
                                compute::hip::functional::loop_accumulate<Red, F, In...> const& b) {
    return for_loop_reductions(std::forward<P>(p), v, st, n, b);
}
// several reductions (for_loop.hpp:802-812)
template <typename P, typename Vars, std::size_t N, typename... A>
result_t<P, void> for_loop_body(P&& p, Vars const& v, strides_t<N> const& st, uint64_t n,
                                compute::hip::functional::loop_accumulate_all<A...> const& b) {
    return std::apply(
        [&](A const&... parts) { return for_loop_reductions(std::forward<P>(p), v, st, n, parts...); }, b.parts);
}
template <typename P, typename Vars, std::size_t N, std::size_t Out, typename F, std::size_t In0>
result_t<P, void> for_loop_body(P&& p, Vars const& v, strides_t<N> const& st, uint64_t n,
                                compute::hip::functional::loop_assign<Out, F, In0> const& b) {
    auto in = std::get<In0>(v);
    auto out = std::get<Out>(v);
    using TI = value_t<decltype(in)>;
    using TO = value_t<decltype(out)>;
    using Tr = tr::unary_t<F>;
    using C = tr::compute_t<Tr, F, TI>;
    C s[2] = {};
    Tr::scalars(b.f, s);
    TI const* pin = raw_ptr(in);
    TO* pout = raw_ptr(out);
    return run_elementwise<void>(
        p, in, n,
        [&](auto const& t, uint64_t off, uint64_t cnt) {
            const int64_t o = static_cast<int64_t>(off);
            check(hpxhip_transform_strided(dt<TI>, dt<C>, dt<TO>, Tr::kind, s, pin + o * st[In0], st[In0],
                                           pout + o * st[Out], st[Out], cnt, t.stream()),
                  "for_loop_n");
        },
        [] {});
}
template <typename P, typename Vars, std::size_t N, std::size_t Out, typename F, std::size_t In0, std::size_t In1>
result_t<P, void> for_loop_body(P&& p, Vars const& v, strides_t<N> const& st, uint64_t n,
                                compute::hip::functional::loop_assign<Out, F, In0, In1> const& b) {
    auto in0 = std::get<In0>(v);
    auto in1 = std::get<In1>(v);
    auto out = std::get<Out>(v);
    using TI = value_t<decltype(in0)>;
    static_assert(std::is_same<TI, value_t<decltype(in1)>>::value, "for_loop_n: both inputs need one element type");
    using TO = value_t<decltype(out)>;
    using Tr = tr::binary_t<F>;
    using C = tr::compute_t<Tr, F, TI>;
    C s[2] = {};
    Tr::scalars(b.f, s);
    TI const* p0 = raw_ptr(in0);
    TI const* p1 = raw_ptr(in1);
    TO* pout = raw_ptr(out);
    return run_elementwise<void>(
        p, in0, n,
        [&](auto const& t, uint64_t off, uint64_t cnt) {
            const int64_t o = static_cast<int64_t>(off);
            check(hpxhip_transform_binary_strided(dt<TI>, dt<C>, dt<TO>, Tr::kind, s, p0 + o * st[In0], st[In0],
                                                  p1 + o * st[In1], st[In1], pout + o * st[Out], st[Out], cnt,
                                                  t.stream()),
                  "for_loop_n");
        },
        [] {});
}

// Any other body: body(first + i*stride, induction_k + i*stride_k, ...) on a
// kernel instantiated for it (hipcc only).  Loop variables reach the body as
// raw device pointers, as in for_loop_compute.cu:40-48 (`int* A, int* B, int* C`).
// A generic body with reductions (hipcc only): body(first + i*stride,
// induction_k + i*stride_k, ..., T& view_r, ...) -- every reduction reaches
// the body as a reference to the thread's private view, which starts at the
// reduction's identity (for_loop_reduction.hpp:35-132); the views are
// combined on the device in a fixed order (device_closures.hpp) and folded
// into the live-out variables on the loop's completion.
template <typename V>
auto loop_reduce_arg(V const& x, int64_t stride) {
    if constexpr (is_reduction<V>::value) {
        using T = std::decay_t<decltype(x.identity_)>;
        using Op = std::decay_t<decltype(x.op_)>;
        (void)stride;
        return red_arg<T, Op>{x.identity_, x.op_};
    } else {
        return strided_ptr<std::remove_pointer_t<std::decay_t<decltype(raw_ptr(x))>>>{raw_ptr(x), stride};
    }
}
template <typename P, typename Vars, std::size_t N, typename B, std::size_t... I>
result_t<P, void> for_loop_generic_reduce(P&& p, Vars const& v, strides_t<N> const& st, uint64_t n, B const& body,
                                          std::index_sequence<I...>) {
    auto const& t = target_of(p, std::get<0>(v));
    constexpr std::size_t nred = count_reductions<Vars>(std::index_sequence<I...>{});
    auto slot = t.make_result_slot();
    void* ws = nullptr;
    check(hpxhip_stream_scratch(t.stream(), kLoopReduceMaxBlocks * nred * sizeof(uint64_t), &ws),
          "for_loop reduction scratch");
    auto* partials = static_cast<uint64_t*>(ws);
    device_loop_reduce(t, body, n, partials, static_cast<uint64_t*>(slot.device()),
                       loop_reduce_arg(std::get<I>(v), st[I])...);
    fetch_slot(t, slot, 8 * nred, "for_loop_n result");
    std::vector<std::function<void(unsigned char const*)>> folds;
    (
        [&] {
            auto const& x = std::get<I>(v);
            if constexpr (is_reduction<std::decay_t<decltype(x)>>::value) {
                using T = std::decay_t<decltype(x.identity_)>;
                T* var = &x.var_;
                auto op = x.op_;
                folds.push_back([var, op](unsigned char const* b) {
                    T view;
                    std::memcpy(&view, b, sizeof(T));
                    *var = op(*var, view);
                });
            }
        }(),
        ...);
    return finish_slot<void>(p, t, std::move(slot), [](unsigned char const*) {},
                             [folds = std::move(folds)](unsigned char const* b) {
                                 for (std::size_t k = 0; k < folds.size(); ++k) folds[k](b + 8 * k);
                             });
}

template <typename P, typename Vars, std::size_t N, typename B, std::size_t... I>
result_t<P, void> for_loop_generic(P&& p, Vars const& v, strides_t<N> const& st, uint64_t n, B const& body,
                                   std::index_sequence<I...> seq) {
    if constexpr ((is_reduction<std::decay_t<std::tuple_element_t<I, Vars>>>::value || ...)) {
        return for_loop_generic_reduce(std::forward<P>(p), v, st, n, body, seq);
    } else {
    auto ptrs = std::make_tuple(raw_ptr(std::get<I>(v))...);
    return run_elementwise<void>(
        p, std::get<0>(v), n,
        [&](auto const& t, uint64_t off, uint64_t cnt) {
            const int64_t o = static_cast<int64_t>(off);
            device_loop(t, body, cnt,
                        strided_ptr<std::remove_pointer_t<std::decay_t<decltype(std::get<I>(ptrs))>>>{
                            std::get<I>(ptrs) + o * st[I], st[I]}...);
        },
        [] {});
    }
}
template <typename Body>
struct is_builtin_body : std::false_type {};
template <std::size_t Out, typename F, std::size_t... In>
struct is_builtin_body<compute::hip::functional::loop_assign<Out, F, In...>> : std::true_type {};
template <std::size_t Red, typename F, std::size_t... In>
struct is_builtin_body<compute::hip::functional::loop_accumulate<Red, F, In...>> : std::true_type {};
template <typename... A>
struct is_builtin_body<compute::hip::functional::loop_accumulate_all<A...>> : std::true_type {};

template <typename P, typename Vars, std::size_t N, typename B,
          typename = std::enable_if_t<!is_builtin_body<std::decay_t<B>>::value>>
result_t<P, void> for_loop_body(P&& p, Vars const& v, strides_t<N> const& st, uint64_t n, B const& body) {
    return for_loop_generic(std::forward<P>(p), v, st, n, body, std::make_index_sequence<N>{});
}
template <typename P, typename It, typename Tuple, std::size_t... I>
auto for_loop_dispatch(P&& p, It first, int64_t first_stride, uint64_t n, Tuple&& args, std::index_sequence<I...>) {
    constexpr std::size_t last = std::tuple_size<std::decay_t<Tuple>>::value - 1;
    auto vars = std::make_tuple(first, loop_var(std::get<I>(args))...);
    strides_t<sizeof...(I) + 1> st{first_stride, loop_stride(std::get<I>(args))...};
    return for_loop_body(std::forward<P>(p), vars, st, n, std::get<last>(args));
}
}  // namespace detail
namespace algo {

// for_loop.hpp:808 for_loop_n(policy, first, size, inductions..., body) with
// a loop_assign body (the C ABI cannot carry arbitrary closures).
template <typename P, typename It, typename Size, typename... Args>
detail::result_t<P, void> for_loop_n(P&& p, It first, Size count, Args&&... args) {
    static_assert(sizeof...(Args) >= 1, "for_loop_n: missing loop body");
    static_assert(detail::is_dev<It> || std::is_pointer<It>::value,
                  "for_loop_n: the loop variable must be a device iterator or a device pointer");
    uint64_t n = count > 0 ? static_cast<uint64_t>(count) : 0;
    return detail::for_loop_dispatch(std::forward<P>(p), first, 1, n, std::forward_as_tuple(args...),
                                     std::make_index_sequence<sizeof...(Args) - 1>{});
}
template <typename P, typename It, typename... Args>
detail::result_t<P, void> for_loop(P&& p, It first, It last, Args&&... args) {
    return for_loop_n(std::forward<P>(p), first, detail::distance(first, last), std::forward<Args>(args)...);
}

// for_loop.hpp:1014 for_loop_n_strided(policy, first, size, stride, args..., f):
// the loop variable advances by `stride` per application, inductions by
// their own stride per application (ordinal position).
template <typename P, typename It, typename Size, typename S, typename... Args>
detail::result_t<P, void> for_loop_n_strided(P&& p, It first, Size count, S stride, Args&&... args) {
    static_assert(sizeof...(Args) >= 1, "for_loop_n_strided: missing loop body");
    static_assert(detail::is_dev<It> || std::is_pointer<It>::value,
                  "for_loop_n_strided: the loop variable must be a device iterator or a device pointer");
    if (stride == 0) throw hpx::exception(HPXHIP_ERROR_INVALID_ARGUMENT, "for_loop_n_strided: zero stride");
    uint64_t n = count > 0 ? static_cast<uint64_t>(count) : 0;
    return detail::for_loop_dispatch(std::forward<P>(p), first, static_cast<int64_t>(stride), n,
                                     std::forward_as_tuple(args...), std::make_index_sequence<sizeof...(Args) - 1>{});
}
// for_loop.hpp:604 for_loop_strided(policy, first, last, stride, args..., f):
// first, first + stride, ... while before last (after it for stride < 0).
template <typename P, typename It, typename S, typename... Args>
detail::result_t<P, void> for_loop_strided(P&& p, It first, It last, S stride, Args&&... args) {
    if (stride == 0) throw hpx::exception(HPXHIP_ERROR_INVALID_ARGUMENT, "for_loop_strided: zero stride");
    const int64_t st = static_cast<int64_t>(stride);
    const uint64_t len = st > 0 ? detail::distance(first, last) : detail::distance(last, first);
    const uint64_t a = static_cast<uint64_t>(st > 0 ? st : -st);
    return for_loop_n_strided(std::forward<P>(p), first, (len + a - 1) / a, stride, std::forward<Args>(args)...);
}

}  // namespace algo
// The public algorithms: each forwards to its definition in namespace algo
// under the error contract above (detail::guarded).
#define HPXHIP_GUARDED_ALGORITHM(name)                                                                     \
    template <typename P, typename... A,                                                                    \
              typename = std::enable_if_t<execution::is_execution_policy<std::decay_t<P>>::value>>          \
    auto name(P&& p, A&&... a)->decltype(algo::name(std::forward<P>(p), std::forward<A>(a)...)) {           \
        using R_ = decltype(algo::name(std::forward<P>(p), std::forward<A>(a)...));                         \
        return detail::guarded<P, R_>([&]() -> R_ { return algo::name(std::forward<P>(p), std::forward<A>(a)...); }); \
    }
HPXHIP_GUARDED_ALGORITHM(for_each)
HPXHIP_GUARDED_ALGORITHM(for_each_n)
HPXHIP_GUARDED_ALGORITHM(fill)
HPXHIP_GUARDED_ALGORITHM(fill_n)
HPXHIP_GUARDED_ALGORITHM(copy)
HPXHIP_GUARDED_ALGORITHM(copy_n)
HPXHIP_GUARDED_ALGORITHM(copy_if)
HPXHIP_GUARDED_ALGORITHM(transform)
HPXHIP_GUARDED_ALGORITHM(reduce)
HPXHIP_GUARDED_ALGORITHM(transform_reduce)
HPXHIP_GUARDED_ALGORITHM(inclusive_scan)
HPXHIP_GUARDED_ALGORITHM(exclusive_scan)
HPXHIP_GUARDED_ALGORITHM(transform_inclusive_scan)
HPXHIP_GUARDED_ALGORITHM(transform_exclusive_scan)
HPXHIP_GUARDED_ALGORITHM(sort)
HPXHIP_GUARDED_ALGORITHM(is_sorted)
HPXHIP_GUARDED_ALGORITHM(sort_by_key)
HPXHIP_GUARDED_ALGORITHM(merge)
HPXHIP_GUARDED_ALGORITHM(for_loop_n)
HPXHIP_GUARDED_ALGORITHM(for_loop)
HPXHIP_GUARDED_ALGORITHM(for_loop_n_strided)
HPXHIP_GUARDED_ALGORITHM(for_loop_strided)
#undef HPXHIP_GUARDED_ALGORITHM

}  // namespace v1
}}  // namespace hpx::parallel

namespace hpx {
// HPX 1.4 also exposes the algorithms through hpx:: (hpx/include/parallel_*.hpp).
using parallel::v1::copy;
using parallel::v1::copy_if;
using parallel::v1::copy_n;
using parallel::v1::exclusive_scan;
using parallel::v1::fill;
using parallel::v1::fill_n;
using parallel::v1::for_each;
using parallel::v1::for_each_n;
using parallel::v1::for_loop;
using parallel::v1::for_loop_n;
using parallel::v1::for_loop_n_strided;
using parallel::v1::for_loop_strided;
using parallel::v1::induction;
using parallel::v1::reduction;
using parallel::v1::reduction_bit_and;
using parallel::v1::reduction_bit_or;
using parallel::v1::reduction_bit_xor;
using parallel::v1::reduction_max;
using parallel::v1::reduction_min;
using parallel::v1::reduction_multiplies;
using parallel::v1::reduction_plus;
using parallel::v1::merge;
using parallel::v1::inclusive_scan;
using parallel::v1::reduce;
using parallel::v1::is_sorted;
using parallel::v1::sort;
using parallel::v1::sort_by_key;
using parallel::v1::transform;
using parallel::v1::transform_exclusive_scan;
using parallel::v1::transform_inclusive_scan;
using parallel::v1::transform_reduce;
}  // namespace hpx

// the segmented algorithms' definitions (they call back into the above)
#include <hpx/parallel/segmented_algorithms.hpp>
