// hpx/lcos/local/sliding_semaphore.hpp -- hpx::lcos::local::sliding_semaphore
// (hpx/lcos/local/sliding_semaphore.hpp, detail/sliding_semaphore.hpp):
// wait(upper) blocks while upper - max_difference > lower, where lower is the
// largest value passed to signal().  1d_stencil_4.cpp:156-186 uses it to bound
// the depth of the dataflow tree it builds ahead of the computation.  Host
// threads here (std::mutex / condition_variable): the signal comes from a
// continuation running on the completion engine.
#pragma once

#include <algorithm>
#include <condition_variable>
#include <cstdint>
#include <mutex>

namespace hpx { namespace lcos { namespace local {

class sliding_semaphore {
public:
    explicit sliding_semaphore(std::int64_t max_difference, std::int64_t lower_limit = 0)
        : max_difference_(max_difference), lower_limit_(lower_limit) {}

    void wait(std::int64_t upper_limit) {
        std::unique_lock<std::mutex> lk(m_);
        cv_.wait(lk, [&] { return !(upper_limit - max_difference_ > lower_limit_); });
    }
    // true (after waiting, which then returns at once) if wait(upper_limit)
    // would not block
    bool try_wait(std::int64_t upper_limit) {
        std::lock_guard<std::mutex> lk(m_);
        return !(upper_limit - max_difference_ > lower_limit_);
    }
    void signal(std::int64_t lower_limit) {
        {
            std::lock_guard<std::mutex> lk(m_);
            lower_limit_ = (std::max)(lower_limit, lower_limit_);
        }
        cv_.notify_all();
    }
    std::int64_t signal_all() {
        std::int64_t l;
        {
            std::lock_guard<std::mutex> lk(m_);
            l = lower_limit_;
        }
        cv_.notify_all();
        return l;
    }

private:
    std::mutex m_;
    std::condition_variable cv_;
    std::int64_t max_difference_;
    std::int64_t lower_limit_;
};

}}}  // namespace hpx::lcos::local
