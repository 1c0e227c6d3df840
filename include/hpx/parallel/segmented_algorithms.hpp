// hpx/parallel/segmented_algorithms.hpp -- the segmented algorithms over
// hpx::partitioned_vector iterators (one process, partitions on HIP targets).
//
//   for_each / fill            segmented_algorithms/for_each.hpp:40-213 (per-segment
//                              dispatch, no combine)
//   transform (unary, binary)  segmented_algorithms/transform.hpp
//   reduce / transform_reduce  segmented_algorithms/reduce.hpp:112-209,
//                              detail/reduce.hpp:31-63: S_j per segment (no init),
//                              then init (op) S_0 (op) ... in segment order
//   inclusive/exclusive scans  segmented_algorithms/detail/scan.hpp:527-696:
//                              1. segment totals, 2. carries in segment order
//                              (carry_{j+1} = carry_j (op) S_j), 3. each segment
//                              scanned with init = its carry
//   copy                       partitioned_vector <-> partitioned_vector / host range
//
// Every segment's work runs on its partition's target stream as a task
// (par(task) on the partition's device iterators), so segments on different
// GPUs run concurrently.  The per-segment results of reduce and the scans
// (segment totals, carries) stay on the devices: they are peer-copied to the
// first segment's target, folded there in segment order (hpxhip_fold /
// hpxhip_fold_exclusive) and the carries copied back, all stream-ordered with
// events -- no host round trip, so a task policy returns before the device
// work is done and its future completes from the streams.
#pragma once

#include <hpx/parallel/algorithms.hpp>
#include <hpx/parallel/segmented_fwd.hpp>

#include <algorithm>
#include <limits>
#include <vector>

namespace hpx { namespace parallel { inline namespace v1 { namespace segmented_detail {

namespace ex = hpx::parallel::execution;

template <typename P>
constexpr bool task_policy = execution::is_async_execution_policy<typename std::decay<P>::type>::value;

// A segment of [a, b) inside partition `part`, as local indices [lo, hi).
struct segment {
    std::size_t part, lo, hi;
};

template <typename PV>
std::vector<segment> segments_of(PV& pv, std::size_t a, std::size_t b) {
    std::vector<segment> s;
    if (a >= b) return s;
    for (std::size_t j = pv.partition_of(a); j < pv.get_num_partitions(); ++j) {
        auto const& p = pv.get_partition(j);
        if (p.first >= b) break;
        const std::size_t lo = std::max(a, p.first), hi = std::min(b, p.last);
        if (hi > lo) s.push_back(segment{j, lo - p.first, hi - p.first});
    }
    return s;
}

template <typename It>
std::size_t index_of(It const& it) {
    return it.index();
}

// The identity of a reduction operator (the segment totals S_j carry no
// init, detail/reduce.hpp:43-62; seeding a device reduction with the
// identity gives the same value).  -0.0 for floating-point plus: exactly
// neutral, also for -0.0.
template <typename T, typename Op>
T identity_of() {
    constexpr int k = compute::hip::traits::binop_t<Op>::kind;
    if constexpr (k == HPXHIP_PLUS) return std::is_floating_point<T>::value ? T(-0.0) : T(0);
    else if constexpr (k == HPXHIP_MULTIPLIES) return T(1);
    else if constexpr (k == HPXHIP_MIN)
        return std::numeric_limits<T>::has_infinity ? std::numeric_limits<T>::infinity() : std::numeric_limits<T>::max();
    else if constexpr (k == HPXHIP_MAX)
        return std::numeric_limits<T>::has_infinity ? -std::numeric_limits<T>::infinity()
                                                    : std::numeric_limits<T>::lowest();
    else if constexpr (k == HPXHIP_BIT_AND) return static_cast<T>(~T(0));
    else return T(0);
}

template <typename R, typename P, typename Fut, typename Fn>
typename util::detail::algorithm_result<P, R>::type finish(std::vector<Fut>&& fs, Fn&& fn) {
    if constexpr (task_policy<P>) {
        return hpx::when_all(std::move(fs)).then([fn = std::forward<Fn>(fn)](auto& all) mutable -> R {
            auto v = all.get();
            for (auto& f : v) f.get();  // rethrows a segment's error
            return fn();
        });
    } else {
        for (auto& f : fs) f.get();
        if constexpr (std::is_void<R>::value) fn();
        else return fn();
    }
}

template <typename PV>
void require_same_layout(PV const& a, std::size_t ia, PV const& b, std::size_t ib, char const* what) {
    bool same = a.size() == b.size() && a.get_num_partitions() == b.get_num_partitions() && ia == ib;
    for (std::size_t j = 0; same && j < a.get_num_partitions(); ++j)
        same = a.get_partition(j).target.device() == b.get_partition(j).target.device();
    if (!same)
        throw hpx::exception(HPXHIP_ERROR_UNSUPPORTED,
                             std::string(what) + ": the partitioned_vectors must be laid out alike (same size, "
                                                 "partitions and targets, same position)");
}

// ------------------------------------------------------------- for_each
template <typename P, typename It, typename F>
typename util::detail::algorithm_result<P, It>::type for_each(P&&, It first, It last, F&& f) {
    auto& pv = first.container();
    using LI = typename std::decay<decltype(pv.get_partition(0).data->begin())>::type;
    std::vector<hpx::future<LI>> fs;
    for (auto const& s : segments_of(pv, index_of(first), index_of(last))) {
        auto& d = *pv.get_partition(s.part).data;
        fs.push_back(hpx::parallel::for_each(ex::par(ex::task), d.begin() + s.lo, d.begin() + s.hi, f));
    }
    return finish<It, P>(std::move(fs), [last] { return last; });
}

template <typename P, typename It, typename T>
typename util::detail::algorithm_result<P, void>::type fill(P&&, It first, It last, T const& value) {
    auto& pv = first.container();
    std::vector<hpx::future<void>> fs;
    for (auto const& s : segments_of(pv, index_of(first), index_of(last))) {
        auto& d = *pv.get_partition(s.part).data;
        fs.push_back(hpx::parallel::fill(ex::par(ex::task), d.begin() + s.lo, d.begin() + s.hi, value));
    }
    return finish<void, P>(std::move(fs), [] {});
}

// ------------------------------------------------------------ transform
template <typename P, typename In, typename Out, typename F>
typename util::detail::algorithm_result<P, util::tagged_pair<In, Out>>::type transform(P&&, In first, In last,
                                                                                      Out dest, F&& f) {
    using R = util::tagged_pair<In, Out>;
    auto& pv = first.container();
    auto& pd = dest.container();
    require_same_layout(pv, index_of(first), pd, index_of(dest), "segmented transform");
    using LO = typename std::decay<decltype(pd.get_partition(0).data->begin())>::type;
    using LI = typename std::decay<decltype(pv.get_partition(0).data->begin())>::type;
    std::vector<hpx::future<util::tagged_pair<LI, LO>>> fs;
    for (auto const& s : segments_of(pv, index_of(first), index_of(last))) {
        auto& d = *pv.get_partition(s.part).data;
        auto& o = *pd.get_partition(s.part).data;
        fs.push_back(hpx::parallel::transform(ex::par(ex::task), d.begin() + s.lo, d.begin() + s.hi, o.begin() + s.lo, f));
    }
    Out end = dest + (last - first);
    return finish<R, P>(std::move(fs), [last, end] { return R{last, end}; });
}

template <typename P, typename In1, typename In2, typename Out, typename F>
typename util::detail::algorithm_result<P, util::tagged_tuple<In1, In2, Out>>::type transform_binary(
    P&&, In1 first1, std::size_t n, In2 first2, Out dest, F&& f) {
    using R = util::tagged_tuple<In1, In2, Out>;
    auto& pv = first1.container();
    auto& p2 = first2.container();
    auto& pd = dest.container();
    require_same_layout(pv, index_of(first1), p2, index_of(first2), "segmented transform");
    require_same_layout(pv, index_of(first1), pd, index_of(dest), "segmented transform");
    using L1 = typename std::decay<decltype(pv.get_partition(0).data->begin())>::type;
    using L2 = typename std::decay<decltype(p2.get_partition(0).data->begin())>::type;
    using LO = typename std::decay<decltype(pd.get_partition(0).data->begin())>::type;
    std::vector<hpx::future<util::tagged_tuple<L1, L2, LO>>> fs;
    const std::size_t a = index_of(first1);
    for (auto const& s : segments_of(pv, a, a + n)) {
        auto& d1 = *pv.get_partition(s.part).data;
        auto& d2 = *p2.get_partition(s.part).data;
        auto& o = *pd.get_partition(s.part).data;
        fs.push_back(hpx::parallel::transform(ex::par(ex::task), d1.begin() + s.lo, d1.begin() + s.hi,
                                              d2.begin() + s.lo, o.begin() + s.lo, f));
    }
    const auto d = static_cast<std::ptrdiff_t>(n);
    In1 e1 = first1 + d;
    In2 e2 = first2 + d;
    Out eo = dest + d;
    return finish<R, P>(std::move(fs), [e1, e2, eo] { return R{e1, e2, eo}; });
}

// ------------------------------------------------- segment totals on device
// Segment j's total S_j = id (op) conv(x) ... is reduced on its partition's
// target into a result slot there and copied (peer copy across GPUs) into
// totals[j] of a block on the first segment's target t0, whose stream then
// waits for every segment -- nothing travels through the host.
template <typename V, typename PV, typename Op, typename Conv>
struct segment_totals {
    std::vector<segment> segs;
    compute::hip::target const* t0 = nullptr;
    compute::hip::detail::device_pool* pool0 = nullptr;
    compute::hip::detail::device_pool::block_ref blk{};
    std::vector<compute::hip::result_slot> slots;  // per segment: [0] total, [16] carry

    V* totals() const { return static_cast<V*>(blk.dev); }
    V* carries() const { return reinterpret_cast<V*>(static_cast<char*>(blk.dev) + 16 * ((segs.size() * sizeof(V) + 15) / 16)); }

    segment_totals(PV& pv, std::size_t a, std::size_t b, Op const& op, Conv const& conv) : segs(segments_of(pv, a, b)) {
        namespace hd = compute::hip::detail;
        if (segs.empty()) return;
        t0 = &pv.get_partition(segs[0].part).target;
        pool0 = &hd::device_pool::get(t0->device());
        const std::size_t nseg = segs.size();
        blk = pool0->acquire_block(16 * ((nseg * sizeof(V) + 15) / 16) + (nseg + 1) * sizeof(V));
        const V id = identity_of<V, typename std::decay<Op>::type>();
        for (std::size_t j = 0; j < nseg; ++j) {
            auto const& s = segs[j];
            auto& part = pv.get_partition(s.part);
            auto const& tj = part.target;
            slots.push_back(tj.make_result_slot());
            detail::reduce_into<V>(tj, part.data->data() + s.lo, s.hi - s.lo, id, op, conv, slots[j].device());
            copy_value(totals() + j, *t0, slots[j].device(), tj, tj.stream());
            hd::stream_after(t0->stream(), tj.stream());
        }
    }
    // dst (on `dt`'s device) <- src (on `st`'s device), sizeof(V) bytes on `s`
    static void copy_value(void* dst, compute::hip::target const& dt, void const* src, compute::hip::target const& st,
                           hpxhip_stream s) {
        namespace hd = compute::hip::detail;
        if (dt.device() == st.device())
            hd::check(hpxhip_memcpy_async(dst, src, sizeof(V), HPXHIP_D2D, s), "segment value copy");
        else
            hd::check(hpxhip_memcpy_peer_async(dst, dt.device(), src, st.device(), sizeof(V), s),
                      "segment value peer copy");
    }
    // the block returns to its pool once `s` has passed the work queued so far
    void release_block_after(hpxhip_stream s) {
        auto* pool = pool0;
        auto b = blk;
        compute::hip::detail::on_stream_done(s, [pool, b] { pool->release_block(b); });
    }
};

// --------------------------------------------------------------- reduce
// segmented_algorithms/reduce.hpp:112-209: S_j per segment (no init), then
// init (op) S_0 (op) ... in segment order -- folded on t0's device
// (hpxhip_fold), the value returned through a result slot.
template <typename T, typename P, typename It, typename Op, typename Conv>
typename util::detail::algorithm_result<P, T>::type reduce(P&& p, It first, It last, T init, Op&& op, Conv&& conv) {
    auto& pv = first.container();
    using PV = typename std::decay<decltype(pv)>::type;
    static_assert(compute::hip::traits::is_binop<Op>,
                  "segmented reduce: the segment-order combine runs on the device with a built-in operator");
    segment_totals<T, PV, Op, Conv> st(pv, index_of(first), index_of(last), op, conv);
    if (st.segs.empty()) {
        if constexpr (task_policy<P>) return hpx::make_ready_future(init);
        else return init;
    }
    auto const& t0 = *st.t0;
    auto slot = t0.make_result_slot();
    compute::hip::detail::check(hpxhip_fold(detail::dt<T>, compute::hip::traits::binop_t<Op>::kind, &init, st.totals(),
                                            st.segs.size(), slot.device(), t0.stream()),
                                "segmented reduce fold");
    detail::fetch_slot(t0, slot, sizeof(T), "segmented reduce result");
    st.release_block_after(t0.stream());
    for (std::size_t j = 0; j < st.segs.size(); ++j)  // each slot returns to its pool on its own stream
        pv.get_partition(st.segs[j].part).target.template async_result<void>([](unsigned char const*) {},
                                                                              std::move(st.slots[j]));
    return detail::finish_slot<T>(p, t0, std::move(slot), detail::load_value<T>{});
}

// ----------------------------------------------------------------- scans
// segmented_algorithms/detail/scan.hpp:527-696: 1. segment totals, 2. the
// carries in segment order (carry_0 = init, carry_{j+1} = carry_j (op) S_j:
// hpxhip_fold_exclusive on t0), 3. each segment scanned on its own target
// from its carry, read on the device (hpxhip_scan's prefix).  All of it is
// queued without a host round trip; under a task policy the future is ready
// when every segment's scan is.
template <typename P, typename In, typename Out, typename Op, typename Conv, typename T>
typename util::detail::algorithm_result<P, Out>::type scan(P&&, In first, In last, Out dest, Op&& op, Conv&& conv,
                                                          T init, bool inclusive) {
    namespace hd = compute::hip::detail;
    auto& pv = first.container();
    auto& pd = dest.container();
    require_same_layout(pv, index_of(first), pd, index_of(dest), "segmented scan");
    using PV = typename std::decay<decltype(pv)>::type;
    using V = typename PV::value_type;
    static_assert(compute::hip::traits::is_binop<Op>,
                  "segmented scan: the carries are folded on the device with a built-in operator");
    Out end = dest + (last - first);
    segment_totals<V, PV, Op, Conv> st(pv, index_of(first), index_of(last), op, conv);
    if (st.segs.empty()) {
        if constexpr (task_policy<P>) return hpx::make_ready_future(end);
        else return end;
    }
    auto const& t0 = *st.t0;
    const V iv = static_cast<V>(init);
    hd::check(hpxhip_fold_exclusive(detail::dt<V>, compute::hip::traits::binop_t<Op>::kind, &iv, st.totals(),
                                    st.segs.size(), st.carries(), t0.stream()),
              "segmented scan carries");
    std::vector<hpx::future<void>> fs;
    for (std::size_t j = 0; j < st.segs.size(); ++j) {
        auto const& s = st.segs[j];
        auto& part = pv.get_partition(s.part);
        auto const& tj = part.target;
        V* carry = reinterpret_cast<V*>(static_cast<char*>(st.slots[j].device()) + 16);
        hd::stream_after(tj.stream(), t0.stream());
        st.copy_value(carry, tj, st.carries() + j, t0, tj.stream());
        auto& o = *pd.get_partition(s.part).data;
        detail::scan_into(tj, part.data->data() + s.lo, o.data() + s.lo, s.hi - s.lo, op, conv, iv, carry, inclusive);
        hd::stream_after(t0.stream(), tj.stream());  // t0 releases the carries block after every copy
        fs.push_back(tj.template async_result<void>([](unsigned char const*) {}, std::move(st.slots[j])));
    }
    st.release_block_after(t0.stream());
    if constexpr (task_policy<P>) {
        return hpx::when_all(std::move(fs)).then([end](auto& all) {
            for (auto& f : all.get()) f.get();  // rethrows a segment's error
            return end;
        });
    } else {
        for (auto& f : fs) f.get();
        return end;
    }
}

// ------------------------------------------------------------------ copy
template <typename P, typename In, typename Out>
typename util::detail::algorithm_result<P, util::tagged_pair<In, Out>>::type copy(P&&, In first, In last,
                                                                                 Out dest) {
    using R = util::tagged_pair<In, Out>;
    const auto n = last - first;
    Out end = dest + n;
    if constexpr (is_segmented_iterator<In>::value && is_segmented_iterator<Out>::value) {
        auto& pv = first.container();
        auto& pd = dest.container();
        require_same_layout(pv, index_of(first), pd, index_of(dest), "segmented copy");
        using LI = typename std::decay<decltype(pv.get_partition(0).data->begin())>::type;
        using LO = typename std::decay<decltype(pd.get_partition(0).data->begin())>::type;
        std::vector<hpx::future<util::tagged_pair<LI, LO>>> fs;
        for (auto const& s : segments_of(pv, index_of(first), index_of(last))) {
            auto& d = *pv.get_partition(s.part).data;
            auto& o = *pd.get_partition(s.part).data;
            fs.push_back(hpx::parallel::copy(ex::par(ex::task), d.begin() + s.lo, d.begin() + s.hi, o.begin() + s.lo));
        }
        return finish<R, P>(std::move(fs), [last, end] { return R{last, end}; });
    } else if constexpr (is_segmented_iterator<In>::value) {  // partitioned_vector -> host range
        auto& pv = first.container();
        using LI = typename std::decay<decltype(pv.get_partition(0).data->begin())>::type;
        std::vector<hpx::future<util::tagged_pair<LI, Out>>> fs;
        const std::size_t a = index_of(first);
        for (auto const& s : segments_of(pv, a, index_of(last))) {
            auto const& part = pv.get_partition(s.part);
            auto& d = *part.data;
            fs.push_back(hpx::parallel::copy(ex::par(ex::task), d.begin() + s.lo, d.begin() + s.hi,
                                             dest + static_cast<std::ptrdiff_t>(part.first + s.lo - a)));
        }
        return finish<R, P>(std::move(fs), [last, end] { return R{last, end}; });
    } else {  // host range -> partitioned_vector
        auto& pd = dest.container();
        using LO = typename std::decay<decltype(pd.get_partition(0).data->begin())>::type;
        std::vector<hpx::future<util::tagged_pair<In, LO>>> fs;
        const std::size_t a = index_of(dest);
        for (auto const& s : segments_of(pd, a, a + static_cast<std::size_t>(n))) {
            auto const& part = pd.get_partition(s.part);
            auto& o = *part.data;
            const auto off = static_cast<std::ptrdiff_t>(part.first + s.lo - a);
            fs.push_back(hpx::parallel::copy(ex::par(ex::task), first + off,
                                             first + off + static_cast<std::ptrdiff_t>(s.hi - s.lo), o.begin() + s.lo));
        }
        return finish<R, P>(std::move(fs), [last, end] { return R{last, end}; });
    }
}

}}}}  // namespace hpx::parallel::v1::segmented_detail
