// hpx/compute/hip/concurrent_executor.hpp -- hpx::compute::hip::concurrent_executor,
// the HIP counterpart of hpx/compute/cuda/concurrent_executor.hpp:29-234.
//
// The reference keeps one cuda::default_executor (own target copy, own
// stream) per host NUMA target and round-robins work over them (:44-57,
// :118-199); STREAM's GPU path runs on it (stream.cpp:428-453).  Here the
// executor owns `num_streams` default_executors on one device; there is no
// host block_executor hop (the launches are asynchronous already, so they
// are issued from the calling thread).
//
// concurrent_executor_parameters (concurrent_executor_parameters.hpp:19-27):
// chunk = ceil(num_tasks / cores) with cores = processing_units_count() =
// the number of streams.  The data-parallel algorithms honour it for the
// elementwise ones (for_each, fill, copy, transform, for_loop): the range is
// cut into one chunk per stream and each chunk's kernel runs on its own
// stream.  Reductions, scans, copy_if, sort and merge are single-kernel
// algorithms and run on the first stream.
#pragma once

#include <hpx/compute/hip.hpp>
#include <hpx/compute/hip/default_executor.hpp>
#include <hpx/parallel/execution.hpp>

#include <algorithm>
#include <array>
#include <atomic>
#include <cstddef>
#include <iterator>
#include <utility>
#include <vector>

namespace hpx { namespace compute { namespace hip {

struct concurrent_executor_parameters {
    template <typename Executor, typename F>
    std::size_t get_chunk_size(Executor&, F&&, std::size_t cores, std::size_t num_tasks) const {
        return (num_tasks + cores - 1) / cores;
    }
};

class concurrent_executor {
    std::vector<default_executor> execs_;
    mutable std::atomic<std::size_t> current_{0};

    default_executor const& next() const { return execs_[++current_ % execs_.size()]; }

public:
    using executor_parameters_type = concurrent_executor_parameters;
    using execution_category = parallel::execution::parallel_execution_tag;

    // :44-57: one executor (target copy with its own stream) per slot, streams
    // created eagerly.
    explicit concurrent_executor(hip::target const& t, std::size_t num_streams = 4) {
        if (num_streams == 0) throw hpx::exception(HPXHIP_ERROR_INVALID_ARGUMENT, "concurrent_executor: no streams");
        execs_.reserve(num_streams);
        for (std::size_t i = 0; i != num_streams; ++i) {
            hip::target ti(t.device());
            (void)ti.stream();
            execs_.emplace_back(ti);
        }
    }
    // :59-90: copies share nothing but the device (each copy of a target has
    // its own stream); the round-robin counter restarts.
    concurrent_executor(concurrent_executor const& o) : execs_(o.execs_) {}
    concurrent_executor(concurrent_executor&& o) noexcept : execs_(std::move(o.execs_)), current_(o.current_.load()) {}
    concurrent_executor& operator=(concurrent_executor const& o) {
        if (this != &o) {
            execs_ = o.execs_;
            current_ = 0;
        }
        return *this;
    }

    bool operator==(concurrent_executor const& rhs) const noexcept { return execs_ == rhs.execs_; }
    bool operator!=(concurrent_executor const& rhs) const noexcept { return !(*this == rhs); }

    std::size_t processing_units_count() const { return execs_.size(); }
    hip::target const& context() const noexcept { return execs_.front().target(); }
    // the first stream's target: where the single-kernel algorithms run
    hip::target const& target() const { return execs_.front().target(); }
    std::vector<default_executor> const& executors() const { return execs_; }

    template <typename F, typename... Ts>
    void post(F&& f, Ts&&... ts) const {
        next().post(std::forward<F>(f), std::forward<Ts>(ts)...);
    }
    template <typename F, typename... Ts>
    hpx::future<void> async_execute(F&& f, Ts&&... ts) const {
        return next().async_execute(std::forward<F>(f), std::forward<Ts>(ts)...);
    }
    template <typename F, typename... Ts>
    void sync_execute(F&& f, Ts&&... ts) const {
        next().sync_execute(std::forward<F>(f), std::forward<Ts>(ts)...);
    }
    // :173-199 with concurrent_executor_parameters (chunk = ceil(n / streams)):
    // the shape is cut into one chunk per stream, each chunk one bulk launch
    // on its own stream; nothing waits for the device.  As in the reference
    // (one async_execute per element, :171-193) the result holds one future
    // per shape element: the elements of a chunk share its future.
    template <typename F, typename Shape, typename... Ts>
    std::vector<hpx::future<void>> bulk_async_execute(F&& f, Shape const& shape, Ts&&... ts) const {
        std::vector<hpx::future<void>> result;
        auto chunks = bulk_chunks(f, shape, ts...);
        std::size_t total = 0;
        for (auto const& c : chunks) total += c.second;
        result.reserve(total);
        for (auto& c : chunks)
            for (std::size_t i = 0; i < c.second; ++i) result.push_back(hpx::future<void>(c.first.shared()));
        return result;
    }
    template <typename F, typename Shape, typename... Ts>
    void bulk_sync_execute(F&& f, Shape const& shape, Ts&&... ts) const {
        for (auto& c : bulk_chunks(f, shape, ts...)) c.first.get();
    }

private:
    // (future of the chunk's launch, elements in the chunk) per chunk
    template <typename F, typename Shape, typename... Ts>
    std::vector<std::pair<hpx::future<void>, std::size_t>> bulk_chunks(F const& f, Shape const& shape,
                                                                       Ts const&... ts) const {
        using V = typename std::decay<decltype(*std::begin(shape))>::type;
        std::vector<V> all(std::begin(shape), std::end(shape));
        std::vector<std::pair<hpx::future<void>, std::size_t>> chunks;
        const std::size_t k = execs_.size();
        const std::size_t chunk = concurrent_executor_parameters{}.get_chunk_size(*this, f, k, all.size());
        for (std::size_t off = 0; off < all.size(); off += chunk) {
            auto const& e = next();
            const std::size_t cnt = std::min(chunk, all.size() - off);
            struct range {
                V const* b;
                V const* e;
                V const* begin() const { return b; }
                V const* end() const { return e; }
            };
            e.bulk_launch(f, range{all.data() + off, all.data() + off + cnt}, ts...);  // staged before it returns
            chunks.emplace_back(e.target().get_future(), cnt);
        }
        return chunks;
    }

public:
    void synchronize() const {
        for (auto const& e : execs_) e.target().synchronize();
    }
};

}}}  // namespace hpx::compute::hip

// concurrent_executor.hpp:203-231
namespace hpx { namespace parallel { namespace execution {
template <>
struct executor_execution_category<compute::hip::concurrent_executor> {
    using type = parallel_execution_tag;
};
template <> struct is_one_way_executor<compute::hip::concurrent_executor> : std::true_type {};
template <> struct is_two_way_executor<compute::hip::concurrent_executor> : std::true_type {};
template <> struct is_bulk_one_way_executor<compute::hip::concurrent_executor> : std::true_type {};
template <> struct is_bulk_two_way_executor<compute::hip::concurrent_executor> : std::true_type {};
}}}  // namespace hpx::parallel::execution
