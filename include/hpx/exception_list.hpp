// hpx/exception_list.hpp -- hpx::exception_list, the container of
// exception_ptr through which the parallel algorithms report failures
// (hpx/exception_list.hpp:28-97), and the policy-dependent rethrow rules of
// hpx/parallel/exception_list.hpp:20-165 / handle_local_exceptions.hpp:30-40:
//
//   * std::bad_alloc (hpx::out_of_memory included) passes through unwrapped;
//   * an hpx::exception_list passes through unchanged;
//   * anything else is wrapped: exception_list(current_exception());
//   * synchronous policies throw, task policies return an exceptional future
//     (algorithms.hpp: detail::guarded), par_unseq calls std::terminate.
#pragma once

#include <hpx/exception.hpp>

#include <exception>
#include <list>
#include <mutex>
#include <string>
#include <utility>

namespace hpx {

class exception_list : public hpx::exception {
    using list_type = std::list<std::exception_ptr>;
    list_type exceptions_;
    mutable std::mutex mtx_;

    static int status_of(std::exception_ptr const& e) {
        try {
            if (e) std::rethrow_exception(e);
        } catch (hpx::exception const& x) {
            return x.status;
        } catch (...) {
        }
        return HPXHIP_ERROR_INVALID_ARGUMENT;
    }
    static std::string message_of(list_type const& l) {
        std::string m;
        for (auto const& e : l) {
            try {
                std::rethrow_exception(e);
            } catch (std::exception const& x) {
                m += (m.empty() ? "" : "; ") + std::string(x.what());
            } catch (...) {
                m += (m.empty() ? "" : "; ") + std::string("unknown exception");
            }
        }
        return m.empty() ? std::string("hpx::exception_list") : m;
    }

public:
    using iterator = list_type::const_iterator;

    exception_list() : hpx::exception(HPXHIP_SUCCESS, "hpx::exception_list") {}
    explicit exception_list(std::exception_ptr const& e)
        : hpx::exception(status_of(e), message_of(list_type{e})), exceptions_{e} {}
    explicit exception_list(list_type&& l)
        : hpx::exception(l.empty() ? HPXHIP_SUCCESS : status_of(l.front()), message_of(l)), exceptions_(std::move(l)) {}
    exception_list(exception_list const& o) : hpx::exception(o) {
        std::lock_guard<std::mutex> lk(o.mtx_);
        exceptions_ = o.exceptions_;
    }
    exception_list(exception_list&& o) : hpx::exception(o) {
        std::lock_guard<std::mutex> lk(o.mtx_);
        exceptions_ = std::move(o.exceptions_);
    }
    exception_list& operator=(exception_list const& o) {
        if (this != &o) {
            hpx::exception::operator=(o);
            std::scoped_lock lk(mtx_, o.mtx_);
            exceptions_ = o.exceptions_;
        }
        return *this;
    }
    exception_list& operator=(exception_list&& o) {
        if (this != &o) {
            hpx::exception::operator=(o);
            std::scoped_lock lk(mtx_, o.mtx_);
            exceptions_ = std::move(o.exceptions_);
        }
        return *this;
    }

    void add(std::exception_ptr const& e) {
        std::lock_guard<std::mutex> lk(mtx_);
        if (exceptions_.empty()) status = status_of(e);
        exceptions_.push_back(e);
    }
    std::size_t size() const noexcept {
        std::lock_guard<std::mutex> lk(mtx_);
        return exceptions_.size();
    }
    iterator begin() const noexcept {
        std::lock_guard<std::mutex> lk(mtx_);
        return exceptions_.begin();
    }
    iterator end() const noexcept {
        std::lock_guard<std::mutex> lk(mtx_);
        return exceptions_.end();
    }
    std::string get_message() const { return what(); }
};

namespace detail {
// handle_exception_impl::call(exception_ptr) without the throw: the
// exception_ptr a caller of the algorithm receives for failure e.
inline std::exception_ptr to_algorithm_error(std::exception_ptr const& e) {
    try {
        std::rethrow_exception(e);
    } catch (std::bad_alloc const&) {
        return e;
    } catch (hpx::exception_list const&) {
        return e;
    } catch (...) {
        return std::make_exception_ptr(hpx::exception_list(e));
    }
}
}  // namespace detail

}  // namespace hpx
