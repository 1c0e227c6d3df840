// hpx/lcos/when_all.hpp -- hpx::when_all and hpx::wait_all.
//
//   when_all(Range&&), when_all(first, last), when_all(f1, f2, ...)
//                                           <- hpx/lcos/when_all.hpp
//   wait_all(...)                           <- hpx/lcos/wait_all.hpp
//
// A when_all future holds its input futures (moved in; shared_futures are
// copied) and is ready once every input is.  It completes without the
// completion engine when it is waited for: get() waits on each input in turn
// (an event wait for a device input) and then readies the group; is_ready()
// asks every input.  Only a continuation on the group (then, dataflow) arms
// it: each input then counts the group down from its own completion.
#pragma once

#include <hpx/lcos/future.hpp>

#include <atomic>
#include <iterator>
#include <memory>
#include <tuple>
#include <type_traits>
#include <utility>
#include <vector>

namespace hpx {

namespace lcos { namespace detail {

struct join final : early_completion {
    std::vector<std::shared_ptr<state_base>> ins;
    state_base* st = nullptr;  // the group's state, which owns this object
    std::once_flag armed;
    void wait_and_complete() override {
        for (auto& in : ins) in->wait();
        st->set_ready(0);
    }
    bool try_complete() override {
        for (auto& in : ins)
            if (!in->poll()) return false;
        st->set_ready(0);
        return true;
    }
    void arm(std::shared_ptr<void> keep) override {
        std::call_once(armed, [&] {
            auto self = std::static_pointer_cast<state_base>(keep);
            auto pending = std::make_shared<std::atomic<std::size_t>>(ins.size() + 1);
            auto count_down = [self, pending] {
                if (pending->fetch_sub(1) == 1) self->set_ready(0);
            };
            for (auto& in : ins) state_base::when_ready(in, count_down);
            count_down();
        });
    }
};

// acquire_future: a future is moved out of its argument, a shared_future is
// copied (hpx/traits/acquire_future.hpp)
template <typename F>
typename std::decay<F>::type acquire(F&& f) {
    if constexpr (std::is_lvalue_reference<F>::value && is_plain_future<std::decay_t<F>>::value) return std::move(f);
    else return std::forward<F>(f);
}

template <typename F>
struct is_vector_of_futures : std::false_type {};
template <typename T, typename A>
struct is_vector_of_futures<std::vector<T, A>> : is_future_or_shared<T> {};

// the states of the futures among an argument list: futures, shared_futures
// and vectors of them; anything else is not waited for
template <typename F>
void collect_state(std::vector<std::shared_ptr<state_base>>& out, F const& f) {
    if constexpr (is_future_or_shared<F>::value) {
        if (f.valid()) out.push_back(f.shared());
    } else if constexpr (is_vector_of_futures<F>::value) {
        for (auto const& x : f)
            if (x.valid()) out.push_back(x.shared());
    }
}

template <typename V>
future<V> make_group(V&& value, std::vector<std::shared_ptr<state_base>> ins) {
    auto st = std::make_shared<shared_state<V>>();
    st->value.emplace(std::move(value));
    auto g = std::make_shared<join>();
    g->ins = std::move(ins);
    g->st = st.get();
    st->early = g;
    return future<V>(st);
}
}}  // namespace lcos::detail

// when_all over a range of futures (moved) or shared_futures (copied)
template <typename Range,
          typename = std::enable_if_t<lcos::detail::is_vector_of_futures<std::decay_t<Range>>::value>>
auto when_all(Range&& values) {
    using F = typename std::decay_t<Range>::value_type;
    std::vector<F> v;
    v.reserve(values.size());
    for (auto& f : values) v.push_back(lcos::detail::acquire<decltype(f)>(f));
    std::vector<std::shared_ptr<lcos::detail::state_base>> ins;
    for (auto const& f : v)
        if (f.valid()) ins.push_back(f.shared());
    return lcos::detail::make_group(std::move(v), std::move(ins));
}

// when_all(first, last)
template <typename It, typename = std::enable_if_t<lcos::detail::is_future_or_shared<
                           typename std::iterator_traits<It>::value_type>::value>>
auto when_all(It first, It last) {
    using F = typename std::iterator_traits<It>::value_type;
    std::vector<F> v;
    for (; first != last; ++first) v.push_back(lcos::detail::acquire<decltype(*first)>(*first));
    return when_all(std::move(v));
}

// when_all(f1, f2, ...) -> future<tuple<F1, F2, ...>>
template <typename... Fs,
          typename = std::enable_if_t<(lcos::detail::is_future_or_shared<std::decay_t<Fs>>::value && ...)>>
auto when_all(Fs&&... fs) {
    using Tup = std::tuple<std::decay_t<Fs>...>;
    Tup t(lcos::detail::acquire<Fs>(std::forward<Fs>(fs))...);
    std::vector<std::shared_ptr<lcos::detail::state_base>> ins;
    std::apply([&](auto const&... f) { (lcos::detail::collect_state(ins, f), ...); }, t);
    return lcos::detail::make_group(std::move(t), std::move(ins));
}
inline future<std::tuple<>> when_all() { return make_ready_future(std::tuple<>()); }

// wait_all: returns once every argument (futures, shared_futures, or ranges
// of them) is ready; results and errors stay in the futures
template <typename... Fs>
void wait_all(Fs const&... fs) {
    std::vector<std::shared_ptr<lcos::detail::state_base>> ins;
    (lcos::detail::collect_state(ins, fs), ...);
    for (auto& in : ins) in->wait();
}
template <typename It, typename = std::enable_if_t<lcos::detail::is_future_or_shared<
                           typename std::iterator_traits<It>::value_type>::value>>
void wait_all(It first, It last) {
    for (; first != last; ++first)
        if (first->valid()) first->shared()->wait();
}

}  // namespace hpx
