// hpx/util/unwrapping.hpp -- hpx::util::unwrapping and hpx::util::unwrap.
//
//   unwrapping(f)  <- hpx/util/unwrap.hpp (unwrapping): a callable that calls
//                     f with the values of its future arguments
//   unwrap(f)      <- hpx/util/unwrap.hpp (unwrap): the value of one future
//
// Per argument: future<T> -> T, shared_future<T> -> T const&, a
// future<void> / shared_future<void> is dropped from the argument list,
// vector<future<T>> / vector<shared_future<T>> -> vector<T>; anything else is
// passed through.  A future holding an error rethrows it (into the task that
// called the unwrapped function, so the error lands in its future).
#pragma once

#include <hpx/lcos/future.hpp>
#include <hpx/lcos/when_all.hpp>

#include <functional>
#include <tuple>
#include <type_traits>
#include <utility>
#include <vector>

namespace hpx { namespace util {

namespace detail {
template <typename A>
auto unwrap_arg(A&& a) {
    using D = std::decay_t<A>;
    if constexpr (hpx::lcos::detail::is_future_or_shared<D>::value) {
        using T = typename hpx::lcos::detail::shared_state_of<D>::type;
        if constexpr (std::is_void<T>::value) {
            a.get();
            return std::tuple<>();
        } else if constexpr (hpx::lcos::detail::is_plain_future<D>::value) {
            return std::tuple<T>(a.get());
        } else {
            return std::tuple<T const&>(a.get());
        }
    } else if constexpr (hpx::lcos::detail::is_vector_of_futures<D>::value) {
        using T = typename hpx::lcos::detail::shared_state_of<typename D::value_type>::type;
        if constexpr (std::is_void<T>::value) {
            for (auto& f : a) f.get();
            return std::tuple<>();
        } else {
            std::vector<T> out;
            out.reserve(a.size());
            for (auto& f : a) out.push_back(f.get());
            return std::tuple<std::vector<T>>(std::move(out));
        }
    } else {
        return std::tuple<A&&>(std::forward<A>(a));
    }
}

template <typename F>
struct unwrapped {
    F f;
    template <typename... Ts>
    decltype(auto) operator()(Ts&&... ts) {
        return std::apply(
            [&](auto&&... a) -> decltype(auto) { return std::invoke(f, std::forward<decltype(a)>(a)...); },
            std::tuple_cat(unwrap_arg(std::forward<Ts>(ts))...));
    }
    template <typename... Ts>
    decltype(auto) operator()(Ts&&... ts) const {
        return std::apply(
            [&](auto&&... a) -> decltype(auto) { return std::invoke(f, std::forward<decltype(a)>(a)...); },
            std::tuple_cat(unwrap_arg(std::forward<Ts>(ts))...));
    }
};
}  // namespace detail

template <typename F>
detail::unwrapped<std::decay_t<F>> unwrapping(F&& f) {
    return {std::forward<F>(f)};
}

template <typename Fut, typename = std::enable_if_t<hpx::lcos::detail::is_future_or_shared<std::decay_t<Fut>>::value>>
decltype(auto) unwrap(Fut&& f) {
    return f.get();
}

}}  // namespace hpx::util
