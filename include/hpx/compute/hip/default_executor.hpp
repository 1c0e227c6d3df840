// hpx/compute/hip/default_executor.hpp -- hpx::compute::hip::default_executor,
// the HIP counterpart of hpx/compute/cuda/default_executor.hpp:42-260.
//
// Members (default_executor.hpp:139-230): post / async_execute / sync_execute
// launch one device thread running the closure (<<<1,1>>>, :173-192);
// bulk_async_execute / bulk_sync_execute run f(shape[i], ts...) for every
// element of the shape, one device thread per element, the shape copied to
// the device first (:42-84, :196-215); processing_units_count(), context(),
// executor_parameters_type, operator==.  Traits (:233-260): parallel
// execution category, one-/two-way and bulk one-/two-way.
//
// Device closures need hipcc (see detail/launch.hpp).  The data-parallel
// algorithms of <hpx/parallel/algorithms.hpp> never go through these members:
// they call whole-algorithm kernels on the executor's target (the reference's
// partitioners need future<T> per chunk, which this executor cannot provide,
// SURVEY.md §0.1).
#pragma once

#include <hpx/compute/hip.hpp>
#include <hpx/compute/hip/detail/launch.hpp>
#include <hpx/parallel/execution.hpp>

#include <algorithm>
#include <cstddef>
#include <iterator>
#include <type_traits>
#include <utility>
#include <vector>

namespace hpx { namespace compute { namespace hip {

// default_executor_parameters.hpp:20-28: one chunk covering the whole range.
struct default_executor_parameters {
    template <typename Executor, typename F>
    std::size_t get_chunk_size(Executor&, F&&, std::size_t, std::size_t) const {
        return std::size_t(-1);
    }
};

namespace detail {
#if HPX_HAVE_HIP_DEVICE_CLOSURES
// default_executor.hpp:42-84: f(shape[idx], ts...) per device thread
// (64-bit index, grid-stride, unlike the reference's int block math).
template <typename V>
struct bulk_body {
    template <typename F, typename... Ts>
    __device__ void operator()(F& f, V const* p, uint64_t count, Ts&... ts) const {
        uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
        for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < count; i += stride) f(p[i], ts...);
    }
};
#endif
}  // namespace detail

class default_executor {
    hip::target target_;

public:
    using executor_parameters_type = default_executor_parameters;
    using execution_category = parallel::execution::parallel_execution_tag;

    default_executor() = default;
    // default_executor.hpp:144-146: the executor holds a copy of the target
    // (so its own stream, cuda_target.cpp:203-211).
    explicit default_executor(hip::target const& t) : target_(t) {}

    bool operator==(default_executor const& rhs) const noexcept { return target_ == rhs.target_; }
    bool operator!=(default_executor const& rhs) const noexcept { return !(*this == rhs); }

    hip::target const& context() const noexcept { return target_; }
    hip::target& target() { return target_; }
    hip::target const& target() const { return target_; }
    std::size_t processing_units_count() const { return target_.processing_units(); }

    // :173-177
    template <typename F, typename... Ts>
    void post(F&& f, Ts&&... ts) const {
        detail::launch(target_, 1, 1, std::forward<F>(f), std::forward<Ts>(ts)...);
    }
    // :179-185
    template <typename F, typename... Ts>
    hpx::future<void> async_execute(F&& f, Ts&&... ts) const {
        post(std::forward<F>(f), std::forward<Ts>(ts)...);
        return target_.get_future();
    }
    // :187-192
    template <typename F, typename... Ts>
    void sync_execute(F&& f, Ts&&... ts) const {
        post(std::forward<F>(f), std::forward<Ts>(ts)...);
        target_.synchronize();
    }

    // :194-199 (bulk_launch_helper<Shape>, :42-84): the shape is staged in a
    // pinned block and copied to a device block, both from this device's
    // pools and both returned to them from the stream once the launch has
    // run -- no allocation, free or synchronisation per call.  (Round 2 copied
    // from the caller's pageable std::vector and freed it when the call
    // returned; the stream-ordered H2D could then still be reading it, which
    // is what lost the first shape element.  That version synchronised to
    // hide it.)
    template <typename F, typename Shape, typename... Ts>
    void bulk_launch(F&& f, Shape const& shape, Ts&&... ts) const {
#if HPX_HAVE_HIP_DEVICE_CLOSURES
        using V = typename std::decay<decltype(*std::begin(shape))>::type;
        static_assert(std::is_trivially_copyable<V>::value, "bulk shape elements are copied to the device");
        const uint64_t count = static_cast<uint64_t>(std::distance(std::begin(shape), std::end(shape)));
        if (count == 0) return;
        auto& pool = detail::device_pool::get(target_.device());
        const std::size_t bytes = count * sizeof(V);
        auto hb = pool.acquire_host_block(bytes);
        std::copy(std::begin(shape), std::end(shape), static_cast<V*>(hb.dev));
        auto db = pool.acquire_block(bytes);
        hpxhip_stream s = target_.stream();
        auto give_back = [&pool, hb, db] {
            pool.release_host_block(hb);
            pool.release_block(db);
        };
        int rc = hpxhip_memcpy_async(db.dev, hb.dev, bytes, HPXHIP_H2D, s);
        if (rc != HPXHIP_SUCCESS) {
            give_back();
            hip::detail::check(rc, "bulk_launch shape");
        }
        try {
            detail::launch(target_, detail::flat_grid(count), dim3(256), detail::bulk_body<V>{}, std::forward<F>(f),
                           static_cast<V const*>(db.dev), count, std::forward<Ts>(ts)...);
        } catch (...) {
            detail::on_stream_done(s, give_back);
            throw;
        }
        detail::on_stream_done(s, give_back);
#else
        static_assert(detail::dependent_false<F>, "bulk_launch of a device closure needs hipcc");
        (void)f;
        (void)shape;
#endif
    }
    // :201-209: one future for the whole bulk launch
    template <typename F, typename Shape, typename... Ts>
    std::vector<hpx::future<void>> bulk_async_execute(F&& f, Shape const& shape, Ts&&... ts) const {
        bulk_launch(std::forward<F>(f), shape, std::forward<Ts>(ts)...);
        std::vector<hpx::future<void>> result;
        result.push_back(target_.get_future());
        return result;
    }
    // :211-216
    template <typename F, typename Shape, typename... Ts>
    void bulk_sync_execute(F&& f, Shape const& shape, Ts&&... ts) const {
        bulk_launch(std::forward<F>(f), shape, std::forward<Ts>(ts)...);
        target_.synchronize();
    }
};

}}}  // namespace hpx::compute::hip

// default_executor.hpp:233-260
namespace hpx { namespace parallel { namespace execution {
template <>
struct executor_execution_category<compute::hip::default_executor> {
    using type = parallel_execution_tag;
};
template <> struct is_one_way_executor<compute::hip::default_executor> : std::true_type {};
template <> struct is_two_way_executor<compute::hip::default_executor> : std::true_type {};
template <> struct is_bulk_one_way_executor<compute::hip::default_executor> : std::true_type {};
template <> struct is_bulk_two_way_executor<compute::hip::default_executor> : std::true_type {};
}}}  // namespace hpx::parallel::execution
