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
#include <hpx/compute/hip/functional.hpp>
#include <hpx/parallel/execution.hpp>

#include <algorithm>
#include <array>
#include <cstring>
#include <iterator>
#include <type_traits>

namespace hpx { namespace parallel {
inline namespace v1 {

namespace detail {
namespace hip = hpx::compute::hip;
namespace tr = hpx::compute::hip::traits;
using hip::detail::check;

template <typename It>
constexpr bool is_dev = hip::is_device_iterator<typename std::decay<It>::type>::value;
template <typename It>
using value_t = typename std::iterator_traits<It>::value_type;
template <typename T>
constexpr int dt = hip::dtype_of<T>::value;

template <typename P>
using policy_t = typename std::decay<P>::type;
template <typename P>
constexpr bool is_task = policy_t<P>::is_task;

template <typename P, typename It>
hip::target const& target_of(P const& p, It const& it) {
    if constexpr (policy_t<P>::has_executor) return p.executor().target();
    else return it.target();
}

template <typename P, typename R>
using result_t = typename util::detail::algorithm_result<P, R>::type;

// Finish an algorithm whose device work is queued on t's stream.
template <typename R, typename P, typename Fn>
result_t<P, R> finish(P const&, hip::target const& t, Fn&& fn) {
    if constexpr (is_task<P>) {
        return t.template async_result<R>(std::function<R()>(std::forward<Fn>(fn)));
    } else {
        t.synchronize();
        if constexpr (std::is_void<R>::value) fn();
        else return fn();
    }
}

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

// ------------------------------------------------------------- for_each
template <typename P, typename It, typename F>
detail::result_t<P, It> for_each(P&& p, It first, It last, F&& f) {
    static_assert(detail::is_dev<It>, "for_each: device iterators required");
    using T = detail::value_t<It>;
    using Tr = detail::tr::unary_t<F>;
    auto const& t = detail::target_of(p, first);
    uint64_t n = detail::distance(first, last);
    T s[2] = {};
    Tr::scalars(f, s);
    detail::check(hpxhip_for_each(detail::dt<T>, Tr::kind, s, first.device_ptr(), n, t.stream()), "for_each");
    return detail::finish<It>(p, t, [last] { return last; });
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
    static_assert(detail::is_dev<It>, "fill: device iterators required");
    using V = detail::value_t<It>;
    auto const& t = detail::target_of(p, first);
    V v = static_cast<V>(value);
    detail::check(hpxhip_fill(detail::dt<V>, &v, first.device_ptr(), detail::distance(first, last), t.stream()),
                  "fill");
    return detail::finish<void>(p, t, [] {});
}

template <typename P, typename It, typename Size, typename T>
detail::result_t<P, It> fill_n(P&& p, It first, Size count, T value) {
    static_assert(detail::is_dev<It>, "fill_n: device iterators required");
    using V = detail::value_t<It>;
    auto const& t = detail::target_of(p, first);
    uint64_t n = count > 0 ? static_cast<uint64_t>(count) : 0;
    V v = static_cast<V>(value);
    detail::check(hpxhip_fill(detail::dt<V>, &v, first.device_ptr(), n, t.stream()), "fill_n");
    It end = first + static_cast<std::ptrdiff_t>(n);
    return detail::finish<It>(p, t, [end] { return end; });
}

// ------------------------------------------------------------------ copy
template <typename P, typename In, typename Out>
detail::result_t<P, util::tagged_pair<In, Out>> copy(P&& p, In first, In last, Out dest) {
    using R = util::tagged_pair<In, Out>;
    uint64_t n = detail::distance(first, last);
    if constexpr (detail::is_dev<In> && detail::is_dev<Out>) {
        using T = detail::value_t<In>;
        static_assert(std::is_same<T, detail::value_t<Out>>::value, "copy: element types must match");
        auto const& t = detail::target_of(p, first);
        detail::check(hpxhip_copy(detail::dt<T>, first.device_ptr(), dest.device_ptr(), n, t.stream()), "copy");
        Out end = dest + static_cast<std::ptrdiff_t>(n);
        return detail::finish<R>(p, t, [last, end] { return R{last, end}; });
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
    using Tr = detail::tr::pred_t<F>;
    using R = util::tagged_pair<In, Out>;
    auto const& t = detail::target_of(p, first);
    uint64_t n = detail::distance(first, last);
    T arg = static_cast<T>(Tr::arg(f));
    auto slot = t.result_slot();
    detail::check(hpxhip_copy_if(detail::dt<T>, Tr::kind, &arg, first.device_ptr(), dest.device_ptr(), n,
                                 static_cast<uint64_t*>(slot.first), t.stream(), nullptr, 0),
                  "copy_if");
    detail::check(hpxhip_memcpy_async(slot.second, slot.first, 8, HPXHIP_D2H, t.stream()), "copy_if count");
    void* host = slot.second;
    return detail::finish<R>(p, t, [last, dest, host] {
        uint64_t c;
        std::memcpy(&c, host, 8);
        return R{last, dest + static_cast<std::ptrdiff_t>(c)};
    });
}

// ------------------------------------------------------------- transform
template <typename P, typename In, typename Out, typename F,
          typename = typename std::enable_if<detail::tr::is_unary<F>>::type>
detail::result_t<P, util::tagged_pair<In, Out>> transform(P&& p, In first, In last, Out dest, F&& f) {
    static_assert(detail::is_dev<In> && detail::is_dev<Out>, "transform: device iterators required");
    using TI = detail::value_t<In>;
    using TO = detail::value_t<Out>;
    using Tr = detail::tr::unary_t<F>;
    using C = detail::tr::compute_t<Tr, F, TI>;
    using R = util::tagged_pair<In, Out>;
    auto const& t = detail::target_of(p, first);
    uint64_t n = detail::distance(first, last);
    C s[2] = {};
    Tr::scalars(f, s);
    detail::check(hpxhip_transform(detail::dt<TI>, detail::dt<C>, detail::dt<TO>, Tr::kind, s, first.device_ptr(),
                                   dest.device_ptr(), n, t.stream()),
                  "transform");
    Out end = dest + static_cast<std::ptrdiff_t>(n);
    return detail::finish<R>(p, t, [last, end] { return R{last, end}; });
}

namespace detail {
template <typename P, typename In1, typename In2, typename Out, typename F>
result_t<P, util::tagged_tuple<In1, In2, Out>> transform_binary(P&& p, In1 first1, uint64_t n, In2 first2, Out dest,
                                                                F&& f) {
    static_assert(is_dev<In1> && is_dev<In2> && is_dev<Out>, "transform: device iterators required");
    using T = value_t<In1>;
    static_assert(std::is_same<T, value_t<In2>>::value, "transform: input element types must match");
    using TO = value_t<Out>;
    using Tr = tr::binary_t<F>;
    using C = tr::compute_t<Tr, F, T>;
    using R = util::tagged_tuple<In1, In2, Out>;
    auto const& t = target_of(p, first1);
    C s[2] = {};
    Tr::scalars(f, s);
    check(hpxhip_transform_binary(dt<T>, dt<C>, dt<TO>, Tr::kind, s, first1.device_ptr(), first2.device_ptr(),
                                  dest.device_ptr(), n, t.stream()),
          "transform");
    auto d = static_cast<std::ptrdiff_t>(n);
    In1 e1 = first1 + d;
    In2 e2 = first2 + d;
    Out eo = dest + d;
    return finish<R>(p, t, [e1, e2, eo] { return R{e1, e2, eo}; });
}
}  // namespace detail

template <typename P, typename In1, typename In2, typename Out, typename F,
          typename = typename std::enable_if<!detail::tr::is_unary<F> && detail::is_dev<Out>>::type>
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
namespace detail {
template <typename T, typename P, typename It, typename Op, typename Conv>
result_t<P, T> reduce_impl(P&& p, It first, It last, T init, Op&& op, Conv&& conv) {
    static_assert(is_dev<It>, "reduce: device iterators required");
    using TI = value_t<It>;
    auto const& t = target_of(p, first);
    T s[2] = {};
    tr::unary_t<Conv>::scalars(conv, s);
    auto slot = t.result_slot();
    check(hpxhip_transform_reduce(dt<TI>, dt<T>, tr::binop_t<Op>::kind, tr::unary_t<Conv>::kind, s, &init,
                                  first.device_ptr(), distance(first, last), slot.first, t.stream(), nullptr, 0),
          "transform_reduce");
    check(hpxhip_memcpy_async(slot.second, slot.first, sizeof(T), HPXHIP_D2H, t.stream()), "reduce result");
    void* host = slot.second;
    return finish<T>(p, t, [host] {
        T v;
        std::memcpy(&v, host, sizeof(T));
        return v;
    });
}
}  // namespace detail

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
          typename = typename std::enable_if<detail::is_dev<It> && detail::tr::is_unary<Conv>>::type>
detail::result_t<P, T> transform_reduce(P&& p, It first, It last, T init, Red&& red, Conv&& conv) {
    return detail::reduce_impl<T>(std::forward<P>(p), first, last, init, std::forward<Red>(red),
                                  std::forward<Conv>(conv));
}

namespace detail {
template <typename T, typename P, typename It1, typename It2, typename Red, typename Comb>
result_t<P, T> reduce_binary_impl(P&& p, It1 first1, It1 last1, It2 first2, T init, Red&& red, Comb&& comb) {
    static_assert(is_dev<It1> && is_dev<It2>, "transform_reduce: device iterators required");
    using TI = value_t<It1>;
    static_assert(std::is_same<TI, value_t<It2>>::value, "transform_reduce: input element types must match");
    auto const& t = target_of(p, first1);
    T s[2] = {};
    tr::binary_t<Comb>::scalars(comb, s);
    auto slot = t.result_slot();
    check(hpxhip_transform_reduce_binary(dt<TI>, dt<T>, tr::binop_t<Red>::kind, tr::binary_t<Comb>::kind, s, &init,
                                         first1.device_ptr(), first2.device_ptr(), distance(first1, last1),
                                         slot.first, t.stream(), nullptr, 0),
          "transform_reduce");
    check(hpxhip_memcpy_async(slot.second, slot.first, sizeof(T), HPXHIP_D2H, t.stream()), "reduce result");
    void* host = slot.second;
    return finish<T>(p, t, [host] {
        T v;
        std::memcpy(&v, host, sizeof(T));
        return v;
    });
}
}  // namespace detail

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
namespace detail {
template <typename P, typename In, typename Out, typename Op, typename Conv, typename T>
result_t<P, Out> scan_impl(P&& p, In first, In last, Out dest, Op&& op, Conv&& conv, T init, bool inclusive) {
    static_assert(is_dev<In> && is_dev<Out>, "scan: device iterators required");
    using V = value_t<In>;
    static_assert(std::is_same<V, value_t<Out>>::value, "scan: input and output element types must match");
    auto const& t = target_of(p, first);
    uint64_t n = distance(first, last);
    V s[2] = {};
    tr::unary_t<Conv>::scalars(conv, s);
    V iv = static_cast<V>(init);
    check(hpxhip_scan(dt<V>, tr::binop_t<Op>::kind, inclusive ? 1 : 0, tr::unary_t<Conv>::kind, s, &iv, nullptr,
                      first.device_ptr(), dest.device_ptr(), n, t.stream(), nullptr, 0),
          inclusive ? "inclusive_scan" : "exclusive_scan");
    Out end = dest + static_cast<std::ptrdiff_t>(n);
    return finish<Out>(p, t, [end] { return end; });
}
using ident = hpx::compute::hip::functional::identity;
}  // namespace detail

// inclusive_scan.hpp:288 (op, init) and :320 (init, op)
template <typename P, typename In, typename Out, typename A, typename B>
detail::result_t<P, Out> inclusive_scan(P&& p, In first, In last, Out dest, A&& a, B&& b) {
    if constexpr (detail::tr::is_binop<A>)
        return detail::scan_impl(std::forward<P>(p), first, last, dest, std::forward<A>(a), detail::ident{}, b, true);
    else
        return detail::scan_impl(std::forward<P>(p), first, last, dest, std::forward<B>(b), detail::ident{}, a, true);
}
// inclusive_scan.hpp:409 (init) and :511 (op; init = value_type())
template <typename P, typename In, typename Out, typename A>
detail::result_t<P, Out> inclusive_scan(P&& p, In first, In last, Out dest, A&& a) {
    using V = detail::value_t<In>;
    if constexpr (detail::tr::is_binop<A>)
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
template <typename P, typename It, typename Comp = std::less<>>
detail::result_t<P, It> sort(P&& p, It first, It last, Comp&& = Comp()) {
    static_assert(detail::is_dev<It>, "sort: device iterators required");
    using T = detail::value_t<It>;
    auto const& t = detail::target_of(p, first);
    detail::check(hpxhip_sort(detail::dt<T>, first.device_ptr(), detail::distance(first, last),
                              detail::tr::compare_t<Comp>::descending ? 1 : 0, t.stream(), nullptr, 0),
                  "sort");
    return detail::finish<It>(p, t, [last] { return last; });
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
template <typename P, typename Vars, std::size_t N, std::size_t Red, typename F, std::size_t... In>
result_t<P, void> for_loop_body(P&& p, Vars const& v, strides_t<N> const& st, uint64_t n,
                                compute::hip::functional::loop_accumulate<Red, F, In...> const& b) {
    if (((st[In] != 1) || ...))
        throw hpx::exception(HPXHIP_ERROR_UNSUPPORTED,
                             "for_loop_n: a reduction loop reads its inductions with stride 1 (the transform_reduce "
                             "kernels are contiguous)");
    auto const& red = std::get<Red>(v);
    using T = std::decay_t<decltype(red.identity_)>;
    using Op = std::decay_t<decltype(red.op_)>;
    static_assert(std::is_same<std::decay_t<decltype(red)>, reduction_helper<T, Op>>::value,
                  "loop_accumulate: position Red must name the loop's reduction");
    auto ins = std::make_tuple(std::get<In>(v)...);
    auto in0 = std::get<0>(ins);
    using TI = value_t<decltype(in0)>;
    auto const& t = target_of(p, in0);
    T s[2] = {};
    T init = red.identity_;
    auto slot = t.result_slot();
    if constexpr (sizeof...(In) == 1) {
        tr::unary_t<F>::scalars(b.f, s);
        check(hpxhip_transform_reduce(dt<TI>, dt<T>, tr::binop_t<Op>::kind, tr::unary_t<F>::kind, s, &init,
                                      in0.device_ptr(), n, slot.first, t.stream(), nullptr, 0),
              "for_loop_n");
    } else {
        auto in1 = std::get<1>(ins);
        static_assert(std::is_same<TI, value_t<decltype(in1)>>::value, "for_loop_n: both inputs need one element type");
        tr::binary_t<F>::scalars(b.f, s);
        check(hpxhip_transform_reduce_binary(dt<TI>, dt<T>, tr::binop_t<Op>::kind, tr::binary_t<F>::kind, s, &init,
                                             in0.device_ptr(), in1.device_ptr(), n, slot.first, t.stream(), nullptr, 0),
              "for_loop_n");
    }
    check(hpxhip_memcpy_async(slot.second, slot.first, sizeof(T), HPXHIP_D2H, t.stream()), "for_loop_n result");
    void* host = slot.second;
    T* var = &red.var_;
    Op op = red.op_;
    // exit_iteration (for_loop_reduction.hpp:60-66): fold the view into var
    return finish<void>(p, t, [host, var, op] {
        T view;
        std::memcpy(&view, host, sizeof(T));
        *var = op(*var, view);
    });
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
    auto const& t = target_of(p, in);
    C s[2] = {};
    Tr::scalars(b.f, s);
    check(hpxhip_transform_strided(dt<TI>, dt<C>, dt<TO>, Tr::kind, s, in.device_ptr(), st[In0], out.device_ptr(),
                                   st[Out], n, t.stream()),
          "for_loop_n");
    return finish<void>(p, t, [] {});
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
    auto const& t = target_of(p, in0);
    C s[2] = {};
    Tr::scalars(b.f, s);
    check(hpxhip_transform_binary_strided(dt<TI>, dt<C>, dt<TO>, Tr::kind, s, in0.device_ptr(), st[In0],
                                          in1.device_ptr(), st[In1], out.device_ptr(), st[Out], n, t.stream()),
          "for_loop_n");
    return finish<void>(p, t, [] {});
}
template <typename P, typename It, typename Tuple, std::size_t... I>
auto for_loop_dispatch(P&& p, It first, int64_t first_stride, uint64_t n, Tuple&& args, std::index_sequence<I...>) {
    constexpr std::size_t last = std::tuple_size<std::decay_t<Tuple>>::value - 1;
    auto vars = std::make_tuple(first, loop_var(std::get<I>(args))...);
    strides_t<sizeof...(I) + 1> st{first_stride, loop_stride(std::get<I>(args))...};
    return for_loop_body(std::forward<P>(p), vars, st, n, std::get<last>(args));
}
}  // namespace detail

// for_loop.hpp:808 for_loop_n(policy, first, size, inductions..., body) with
// a loop_assign body (the C ABI cannot carry arbitrary closures).
template <typename P, typename It, typename Size, typename... Args>
detail::result_t<P, void> for_loop_n(P&& p, It first, Size count, Args&&... args) {
    static_assert(sizeof...(Args) >= 1, "for_loop_n: missing loop body");
    static_assert(detail::is_dev<It>, "for_loop_n: the loop variable must be a device iterator");
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
    static_assert(detail::is_dev<It>, "for_loop_n_strided: the loop variable must be a device iterator");
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
using parallel::v1::sort;
using parallel::v1::sort_by_key;
using parallel::v1::transform;
using parallel::v1::transform_exclusive_scan;
using parallel::v1::transform_inclusive_scan;
using parallel::v1::transform_reduce;
}  // namespace hpx
