// hpx/lcos/async.hpp -- hpx::async(f, args...) and hpx::async(policy, f, args...)
// (hpx/lcos/async.hpp): f(args...) runs on the completion engine's thread
// (launch::async, the default), inline (launch::sync) or when the result is
// waited for (launch::deferred); its result, or the error it throws, is
// held by the returned future (a future returned by f is unwrapped).
#pragma once

#include <hpx/lcos/future.hpp>

#include <functional>
#include <memory>
#include <tuple>
#include <type_traits>
#include <utility>

namespace hpx {

template <typename Policy, typename F, typename... Ts,
          typename = std::enable_if_t<hpx::detail::is_launch_policy<std::decay_t<Policy>>::value>>
auto async(Policy p, F&& f, Ts&&... ts) {
    auto args = std::make_shared<std::tuple<std::decay_t<Ts>...>>(std::forward<Ts>(ts)...);
    return lcos::detail::make_task(p, {}, [args, f = std::forward<F>(f)]() mutable {
        return std::apply([&](auto&&... a) { return std::invoke(f, std::move(a)...); }, *args);
    });
}
template <typename F, typename... Ts,
          typename = std::enable_if_t<!hpx::detail::is_launch_policy<std::decay_t<F>>::value>>
auto async(F&& f, Ts&&... ts) {
    return async(launch::async, std::forward<F>(f), std::forward<Ts>(ts)...);
}

}  // namespace hpx
