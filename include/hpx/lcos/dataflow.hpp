// hpx/lcos/dataflow.hpp -- hpx::dataflow.
//
//   dataflow(F, args...), dataflow(policy, F, args...)
//                                   <- hpx/lcos/dataflow.hpp:532 (and the
//                                      frame around it, :95-400)
//
// f(args...) runs once every future among args (futures, shared_futures and
// vectors of them) is ready; the ready futures themselves are passed to f
// (wrap f in hpx::util::unwrapping to receive their values).  The result is
// a future of f's result; a future returned by f is unwrapped, so a
// continuation that launches device work (a hip-executor algorithm under
// par(task)) yields a future that is ready when that work is.  Default
// policy launch::async: f runs on the completion engine's thread (which may
// call HIP) once its inputs complete, or on a thread that waits for the
// result first; nothing blocks the caller of dataflow.
#pragma once

#include <hpx/lcos/future.hpp>
#include <hpx/lcos/when_all.hpp>

#include <functional>
#include <memory>
#include <tuple>
#include <type_traits>
#include <utility>
#include <vector>

namespace hpx {

template <typename Policy, typename F, typename... Ts,
          typename = std::enable_if_t<hpx::detail::is_launch_policy<std::decay_t<Policy>>::value>>
auto dataflow(Policy p, F&& f, Ts&&... ts) {
    auto args = std::make_shared<std::tuple<std::decay_t<Ts>...>>(lcos::detail::acquire<Ts>(std::forward<Ts>(ts))...);
    std::vector<std::shared_ptr<lcos::detail::state_base>> ins;
    std::apply([&](auto const&... a) { (lcos::detail::collect_state(ins, a), ...); }, *args);
    return lcos::detail::make_task(p, std::move(ins), [args, f = std::forward<F>(f)]() mutable {
        return std::apply(
            [&](auto&&... a) { return std::invoke(f, std::move(a)...); }, *args);
    });
}

template <typename F, typename... Ts,
          typename = std::enable_if_t<!hpx::detail::is_launch_policy<std::decay_t<F>>::value>>
auto dataflow(F&& f, Ts&&... ts) {
    return dataflow(launch::async, std::forward<F>(f), std::forward<Ts>(ts)...);
}

}  // namespace hpx
