// hpx/lcos/future.hpp -- hpx::future, hpx::shared_future and the shared
// state behind them, for the MI355X backend's C++ layer.
//
//   hpx::future<T>, future::then, share    <- hpx/lcos/future.hpp
//   hpx::shared_future<T>                  <- hpx/lcos/future.hpp (shared_future)
//   hpx::make_ready_future / exceptional   <- hpx/lcos/future.hpp
//   hpx::launch::{async, sync, deferred}   <- hpx/runtime/launch_policy.hpp
//   completion of device work              <- src/compute/cuda/cuda_target.cpp:97-142
//
// Device work completes through HIP events.  A get() that has to wait
// synchronises on the event recorded behind the work and completes the state
// itself; is_ready() queries it.  Something that must be told without being
// asked -- a continuation (then, dataflow) or a when_all input armed by one --
// registers the event with the process's completion engine: one host thread
// that polls the pending events (hipEventQuery) and runs the continuations,
// HIP calls included.  The reference registers a stream callback per future
// instead (cuda_target.cpp:97-142), whose hand-off costs ~30 us on this
// runtime and whose thread may not call HIP, so a continuation could not
// launch the next kernel from it; polling is the later HPX design
// (hpx::cuda::experimental's event polling) and what this layer uses.
#pragma once

#include <hpxhip.h>
#include <hpx/exception.hpp>
#include <hpx/exception_list.hpp>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstddef>
#include <cstdint>
#include <exception>
#include <functional>
#include <memory>
#include <mutex>
#include <optional>
#include <string>
#include <thread>
#include <tuple>
#include <type_traits>
#include <utility>
#include <vector>

namespace hpx {

namespace compute { namespace hip { namespace detail {
inline void check(int status, char const* what) {
    if (status == HPXHIP_SUCCESS) return;
    std::string msg = std::string(what) + ": " + hpxhip_error_string(status);
    if (status == HPXHIP_ERROR_OUT_OF_MEMORY) throw out_of_memory(msg);
    throw kernel_error(status, msg);
}
inline kernel_error check_noexcept(int status) {
    return kernel_error(status, std::string("hip completion: ") + hpxhip_error_string(status));
}
}}}  // namespace compute::hip::detail

// ------------------------------------------------------------ launch policy
// hpx/runtime/launch_policy.hpp: where a continuation runs.  async: on the
// completion engine's thread once its inputs are ready (or on a thread that
// waits for its result first); sync: on the thread that makes the last input
// ready; deferred: only when its result is waited for.
namespace detail {
struct async_policy {};
struct sync_policy {};
struct deferred_policy {};
template <typename P>
struct is_launch_policy
    : std::integral_constant<bool, std::is_same<P, async_policy>::value || std::is_same<P, sync_policy>::value ||
                                       std::is_same<P, deferred_policy>::value> {};
}  // namespace detail
struct launch {
    static constexpr detail::async_policy async{};
    static constexpr detail::sync_policy sync{};
    static constexpr detail::deferred_policy deferred{};
};

template <typename T>
class future;
template <typename T>
class shared_future;

namespace lcos { namespace detail {

// The completion engine: one host thread per process that polls the HIP
// events of armed device completions and runs posted continuations.  Started
// on first use; while events are pending it polls without sleeping for ~1 ms,
// then in waits of up to 50 us that a new watch or post cuts short.  Its
// callbacks may call HIP (unlike a hipLaunchHostFunc callback).
class engine {
public:
    static engine& get() {
        static engine e;
        return e;
    }
    // fn(status) runs on the engine thread once `ev` has completed (status 0)
    // or reports an error (the HIP status).
    void watch(hpxhip_event ev, std::function<void(int)> fn) {
        std::lock_guard<std::mutex> lk(m_);
        start_locked();
        incoming_.emplace_back(ev, std::move(fn));
        cv_.notify_one();
    }
    void post(std::function<void()> fn) {
        std::lock_guard<std::mutex> lk(m_);
        start_locked();
        posted_.push_back(std::move(fn));
        cv_.notify_one();
    }
    bool on_engine_thread() const { return std::this_thread::get_id() == id_.load(); }
    ~engine() {
        {
            std::lock_guard<std::mutex> lk(m_);
            stop_ = true;
        }
        cv_.notify_all();
        if (th_.joinable()) th_.join();
    }

private:
    engine() = default;
    void start_locked() {
        if (th_.joinable() || stop_) return;
        th_ = std::thread([this] { loop(); });
        id_.store(th_.get_id());
    }
    void loop() {
        id_.store(std::this_thread::get_id());
        std::vector<std::pair<hpxhip_event, std::function<void(int)>>> polled;
        unsigned idle = 0;
        for (;;) {
            std::vector<std::function<void()>> tasks;
            {
                std::unique_lock<std::mutex> lk(m_);
                for (;;) {
                    if (stop_) return;
                    if (!incoming_.empty() || !posted_.empty()) break;
                    if (polled.empty()) {
                        cv_.wait(lk);
                        continue;
                    }
                    if (idle < kSpin) break;
                    const unsigned us = idle - kSpin < 6 ? (1u << (idle - kSpin)) : 50u;
                    cv_.wait_for(lk, std::chrono::microseconds(us));
                    break;
                }
                for (auto& w : incoming_) polled.push_back(std::move(w));
                incoming_.clear();
                tasks.swap(posted_);
            }
            bool progress = !tasks.empty();
            for (auto& t : tasks) run_guarded(t);
            for (std::size_t i = 0; i < polled.size();) {
                const int rc = hpxhip_event_query(polled[i].first);
                if (rc == HPXHIP_ERROR_NOT_READY) {
                    ++i;
                    continue;
                }
                auto fn = std::move(polled[i].second);
                polled[i] = std::move(polled.back());
                polled.pop_back();
                run_guarded([&] { fn(rc); });
                progress = true;
            }
            if (progress) idle = 0;
            else if (idle < kSpin + 64) ++idle;
            if (!progress && idle < kSpin) std::this_thread::yield();
        }
    }
    template <typename F>
    static void run_guarded(F&& f) {
        try {
            f();
        } catch (...) {
            // a continuation's failure is stored in its own future; anything
            // escaping here has no owner left to report to
        }
    }

    static constexpr unsigned kSpin = 1024;
    std::mutex m_;
    std::condition_variable cv_;
    std::vector<std::pair<hpxhip_event, std::function<void(int)>>> incoming_;
    std::vector<std::function<void()>> posted_;
    bool stop_ = false;
    std::thread th_;
    std::atomic<std::thread::id> id_{};
};

// A completion a waiting get() may run itself instead of waiting to be told
// (a device future's event, a task's inputs, a when_all group's members).
struct early_completion {
    virtual void wait_and_complete() = 0;
    virtual bool try_complete() = 0;                          // non-blocking
    virtual void arm(std::shared_ptr<void> keep_state) = 0;  // complete without a waiter
    virtual ~early_completion() = default;
};

struct state_base {
    std::mutex mtx;
    std::condition_variable cv;
    bool ready = false;
    std::exception_ptr exc;
    std::vector<std::function<void()>> continuations;
    std::shared_ptr<early_completion> early;
    // The future of a parallel algorithm under a task policy: its failure is
    // reported as the algorithm's error (bad_alloc or hpx::exception_list,
    // hpx/parallel/exception_list.hpp:81-111), set by parallel::detail::guarded.
    bool algorithm_result = false;

    virtual ~state_base() = default;

    // Continuations run on the thread that readies the state: a waiting
    // get(), or the completion engine -- never a HIP callback thread.
    void set_ready(int status) {
        std::vector<std::function<void()>> conts;
        {
            std::lock_guard<std::mutex> lk(mtx);
            if (ready) return;
            if (status != 0 && !exc) exc = std::make_exception_ptr(compute::hip::detail::check_noexcept(status));
            ready = true;
            conts.swap(continuations);
        }
        cv.notify_all();
        for (auto& c : conts) c();
    }
    void set_exception(std::exception_ptr e) {
        {
            std::lock_guard<std::mutex> lk(mtx);
            if (ready) return;
            exc = std::move(e);
        }
        set_ready(0);
    }
    bool is_ready_now() {
        std::lock_guard<std::mutex> lk(mtx);
        return ready;
    }
    void wait() {
        if (is_ready_now()) return;
        if (early) early->wait_and_complete();
        std::unique_lock<std::mutex> lk(mtx);
        cv.wait(lk, [&] { return ready; });
    }
    bool poll() {
        if (is_ready_now()) return true;
        if (early) early->try_complete();
        return is_ready_now();
    }
    // fn runs once s is ready (at once if it is).  A pending device
    // completion is armed, so fn runs without anyone waiting for s.
    static void when_ready(std::shared_ptr<state_base> const& s, std::function<void()> fn) {
        std::unique_lock<std::mutex> lk(s->mtx);
        if (s->ready) {
            lk.unlock();
            fn();
            return;
        }
        s->continuations.push_back(std::move(fn));
        auto e = s->early;
        lk.unlock();
        if (e) e->arm(s);
    }
};

template <typename T>
struct shared_state : state_base {
    using value_type = typename std::conditional<std::is_void<T>::value, int, T>::type;
    // Result bytes of a device computation, copied out of the pinned result
    // slot by the completion itself: the state owns what get() reads, nothing
    // is borrowed from the target that launched the work.
    alignas(16) unsigned char raw[64] = {};
    std::function<T()> value_fn;  // run once the device work is done, on the first get()
    std::optional<value_type> value;
    std::once_flag evaluated;
    bool retrieved = false;  // a future<T>::get() moved the value out

    // the value (or error) once ready: value_fn runs here, once
    void resolve() {
        wait();
        std::call_once(evaluated, [this] {
            if (!exc && value_fn) {
                try {
                    if constexpr (std::is_void<T>::value) {
                        value_fn();
                        value.emplace(0);
                    } else {
                        value.emplace(value_fn());
                    }
                } catch (...) {
                    exc = std::current_exception();
                }
            }
            if (!exc && !value) {
                if constexpr (std::is_default_constructible<value_type>::value) value.emplace();  // void states
                else exc = std::make_exception_ptr(hpx::exception(HPXHIP_ERROR_INVALID_ARGUMENT, "future: no value"));
            }
            if (exc && algorithm_result) exc = hpx::detail::to_algorithm_error(exc);
        });
    }
};

template <typename T>
struct shared_state_of;
template <typename T>
struct shared_state_of<hpx::future<T>> {
    using type = T;
};
template <typename T>
struct shared_state_of<hpx::shared_future<T>> {
    using type = T;
};

template <typename F>
struct is_future_or_shared : std::false_type {};
template <typename T>
struct is_future_or_shared<hpx::future<T>> : std::true_type {};
template <typename T>
struct is_future_or_shared<hpx::shared_future<T>> : std::true_type {};

template <typename F>
struct is_plain_future : std::false_type {};
template <typename T>
struct is_plain_future<hpx::future<T>> : std::true_type {};

// future<future<U>> -> future<U> (the implicit unwrapping of then/dataflow)
template <typename R>
struct task_result {
    using type = R;
    static constexpr bool nested = false;
};
template <typename U>
struct task_result<hpx::future<U>> {
    using type = U;
    static constexpr bool nested = true;
};
template <typename U>
struct task_result<hpx::shared_future<U>> {
    using type = U;
    static constexpr bool nested = true;
};

// A task: body runs once every input is ready (the frame of
// hpx/lcos/dataflow.hpp:532 and future::then).  Whoever gets there first
// runs it, once: the engine after the inputs were armed (launch::async), the
// thread that readied the last input (launch::sync), or a thread waiting for
// the result (any policy; the only one under launch::deferred).  A body
// that returns a future completes the task when that future does.
template <typename R>
struct task final : early_completion, std::enable_shared_from_this<task<R>> {
    using S = shared_state<R>;
    std::weak_ptr<S> wst;
    std::vector<std::shared_ptr<state_base>> inputs;
    std::function<void(std::shared_ptr<S> const&, task&)> body;
    int policy = 0;  // 0 async, 1 sync, 2 deferred
    std::atomic<bool> claimed{false};
    std::once_flag armed;
    std::mutex inner_m;
    std::shared_ptr<state_base> inner;  // the future a body returned, if any

    void run(std::shared_ptr<S> const& st) {
        if (claimed.exchange(true)) return;
        try {
            body(st, *this);
        } catch (...) {
            st->set_exception(std::current_exception());
        }
    }
    std::shared_ptr<state_base> get_inner() {
        std::lock_guard<std::mutex> lk(inner_m);
        return inner;
    }
    void wait_and_complete() override {
        auto st = wst.lock();
        if (!st) return;
        for (auto& i : inputs) i->wait();
        run(st);
        if (auto in = get_inner()) in->wait();
    }
    bool try_complete() override {
        auto st = wst.lock();
        if (!st) return false;
        if (policy == 2 && !claimed.load()) return false;  // deferred: runs only when waited for
        for (auto& i : inputs)
            if (!i->poll()) return false;
        run(st);
        if (auto in = get_inner()) in->poll();
        return st->is_ready_now();
    }
    void arm(std::shared_ptr<void> keep) override {
        if (policy == 2) return;
        std::call_once(armed, [&] {
            auto st = std::static_pointer_cast<S>(keep);
            auto self = this->shared_from_this();
            auto pending = std::make_shared<std::atomic<std::size_t>>(inputs.size() + 1);
            const int pol = policy;
            auto count_down = [st, self, pending, pol] {
                if (pending->fetch_sub(1) != 1) return;
                // launch::sync runs inline, unless a cascade of inline
                // continuations is already this deep on this thread
                thread_local int depth = 0;
                if (pol == 1 && depth < 64) {
                    ++depth;
                    self->run(st);
                    --depth;
                } else {
                    engine::get().post([st, self] { self->run(st); });
                }
            };
            for (auto& in : inputs) state_base::when_ready(in, count_down);
            count_down();
        });
    }
};

template <typename P>
constexpr int policy_code() {
    if constexpr (std::is_same<P, hpx::detail::sync_policy>::value) return 1;
    else if constexpr (std::is_same<P, hpx::detail::deferred_policy>::value) return 2;
    else return 0;
}

// Build the future of a task over `inputs`.  fn() computes the body's
// result (R, or a future of it).
template <typename Policy, typename Fn>
auto make_task(Policy, std::vector<std::shared_ptr<state_base>> inputs, Fn&& fn);

}}  // namespace lcos::detail

// ------------------------------------------------------------------ future
template <typename T>
class future {
    using state = lcos::detail::shared_state<T>;
    std::shared_ptr<state> st_;
    friend class shared_future<T>;

public:
    using result_type = T;
    future() = default;
    explicit future(std::shared_ptr<state> s) : st_(std::move(s)) {}
    future(future&&) noexcept = default;
    future& operator=(future&&) noexcept = default;
    future(future const&) = delete;
    future& operator=(future const&) = delete;

    bool valid() const { return static_cast<bool>(st_); }
    bool is_ready() const { return st_->poll(); }
    void wait() const { st_->wait(); }
    // A trivially copyable value is copied out and stays readable; any other
    // value is moved out, once (HPX's get() leaves the future without a
    // state: a second get() throws no_state here).
    T get() {
        st_->resolve();
        if (st_->exc) std::rethrow_exception(st_->exc);
        if constexpr (!std::is_void<T>::value) {
            if constexpr (std::is_trivially_copyable<T>::value) {
                return *st_->value;
            } else {
                std::lock_guard<std::mutex> lk(st_->mtx);
                if (st_->retrieved) throw hpx::exception(HPXHIP_ERROR_INVALID_ARGUMENT, "future: no_state (value already retrieved)");
                st_->retrieved = true;
                return std::move(*st_->value);
            }
        }
    }
    bool has_exception() {
        st_->resolve();
        return static_cast<bool>(st_->exc);
    }
    bool has_value() {
        st_->resolve();
        return !st_->exc;
    }
    std::exception_ptr get_exception_ptr() {
        st_->resolve();
        return st_->exc;
    }
    shared_future<T> share() { return shared_future<T>(std::move(*this)); }

    // hpx::future::then: f(future<T>) runs once this future is ready (by
    // default launch::async: on the completion engine, or on a thread that
    // waits for the result first).  A future returned by f is unwrapped.
    // The continuation receives this future (by rvalue when f accepts one).
    template <typename F, typename = std::enable_if_t<!hpx::detail::is_launch_policy<std::decay_t<F>>::value>>
    auto then(F&& f) {
        return then(launch::async, std::forward<F>(f));
    }
    template <typename Policy, typename F,
              typename = std::enable_if_t<hpx::detail::is_launch_policy<std::decay_t<Policy>>::value>>
    auto then(Policy p, F&& f) {
        auto parent = std::static_pointer_cast<lcos::detail::state_base>(st_);
        auto self = std::make_shared<future<T>>(std::move(*this));
        return lcos::detail::make_task(p, {parent}, [self, f = std::forward<F>(f)]() mutable {
            if constexpr (std::is_invocable<F&, future<T>&&>::value) return f(std::move(*self));
            else return f(*self);
        });
    }
    std::shared_ptr<state> const& shared() const { return st_; }
};

// ----------------------------------------------------------- shared_future
// hpx::shared_future: copyable, every copy reads the one shared result.
template <typename T>
class shared_future {
    using state = lcos::detail::shared_state<T>;
    std::shared_ptr<state> st_;

public:
    using result_type = T;
    shared_future() = default;
    explicit shared_future(std::shared_ptr<state> s) : st_(std::move(s)) {}
    shared_future(future<T>&& f) noexcept : st_(std::move(f.st_)) {}
    shared_future& operator=(future<T>&& f) noexcept {
        st_ = std::move(f.st_);
        return *this;
    }
    shared_future(shared_future const&) = default;
    shared_future(shared_future&&) noexcept = default;
    shared_future& operator=(shared_future const&) = default;
    shared_future& operator=(shared_future&&) noexcept = default;

    bool valid() const { return static_cast<bool>(st_); }
    bool is_ready() const { return st_->poll(); }
    void wait() const { st_->wait(); }
    using get_result = typename std::conditional<std::is_void<T>::value, void,
                                                 typename state::value_type const&>::type;
    get_result get() const {
        st_->resolve();
        if (st_->exc) std::rethrow_exception(st_->exc);
        if constexpr (!std::is_void<T>::value) return *st_->value;
    }
    bool has_exception() const {
        st_->resolve();
        return static_cast<bool>(st_->exc);
    }
    bool has_value() const {
        st_->resolve();
        return !st_->exc;
    }
    std::exception_ptr get_exception_ptr() const {
        st_->resolve();
        return st_->exc;
    }
    // f(shared_future<T>) runs once this future is ready; see future::then
    template <typename F, typename = std::enable_if_t<!hpx::detail::is_launch_policy<std::decay_t<F>>::value>>
    auto then(F&& f) const {
        return then(launch::async, std::forward<F>(f));
    }
    template <typename Policy, typename F,
              typename = std::enable_if_t<hpx::detail::is_launch_policy<std::decay_t<Policy>>::value>>
    auto then(Policy p, F&& f) const {
        auto parent = std::static_pointer_cast<lcos::detail::state_base>(st_);
        shared_future self = *this;
        return lcos::detail::make_task(p, {parent}, [self, f = std::forward<F>(f)]() mutable {
            if constexpr (std::is_invocable<F&, shared_future<T>&&>::value) return f(shared_future<T>(self));
            else return f(self);
        });
    }
    std::shared_ptr<state> const& shared() const { return st_; }
};

namespace lcos { namespace detail {
template <typename Policy, typename Fn>
auto make_task(Policy, std::vector<std::shared_ptr<state_base>> inputs, Fn&& fn) {
    using Raw = std::decay_t<decltype(fn())>;
    using TR = task_result<Raw>;
    using R = typename TR::type;
    using S = shared_state<R>;
    auto st = std::make_shared<S>();
    auto t = std::make_shared<task<R>>();
    t->wst = st;
    t->inputs = std::move(inputs);
    t->policy = policy_code<Policy>();
    t->body = [fn = std::forward<Fn>(fn)](std::shared_ptr<S> const& s, task<R>& tk) mutable {
        if constexpr (TR::nested) {
            auto g = fn();
            auto in = g.shared();
            if (!in) throw hpx::exception(HPXHIP_ERROR_INVALID_ARGUMENT, "continuation returned an empty future");
            {
                std::lock_guard<std::mutex> lk(tk.inner_m);
                tk.inner = in;
            }
            state_base::when_ready(in, [s, in] {
                // the inner future's value (its value_fn, e.g. a device
                // result's decode and error-word check, runs here, once)
                in->resolve();
                if (in->exc) {
                    s->set_exception(in->exc);
                    return;
                }
                {
                    std::lock_guard<std::mutex> lk(s->mtx);
                    if constexpr (std::is_void<R>::value) s->value.emplace(0);
                    else if constexpr (!is_plain_future<Raw>::value) s->value.emplace(*in->value);
                    else s->value.emplace(std::move(*in->value));
                }
                s->set_ready(0);
            });
        } else if constexpr (std::is_void<R>::value) {
            fn();
            {
                std::lock_guard<std::mutex> lk(s->mtx);
                s->value.emplace(0);
            }
            s->set_ready(0);
        } else {
            auto v = fn();
            {
                std::lock_guard<std::mutex> lk(s->mtx);
                s->value.emplace(std::move(v));
            }
            s->set_ready(0);
        }
    };
    st->early = t;
    if (t->policy != 2) t->arm(st);  // async / sync: runs without a waiter
    return hpx::future<R>(st);
}
}}  // namespace lcos::detail

template <typename T>
future<typename std::decay<T>::type> make_ready_future(T&& v) {
    using V = typename std::decay<T>::type;
    auto st = std::make_shared<lcos::detail::shared_state<V>>();
    st->value.emplace(std::forward<T>(v));
    st->set_ready(0);
    return future<V>(st);
}
inline future<void> make_ready_future() {
    auto st = std::make_shared<lcos::detail::shared_state<void>>();
    st->value.emplace(0);
    st->set_ready(0);
    return future<void>(st);
}
// hpx/lcos/future.hpp make_exceptional_future: a ready future holding e.
template <typename T>
future<T> make_exceptional_future(std::exception_ptr e) {
    auto st = std::make_shared<lcos::detail::shared_state<T>>();
    st->exc = std::move(e);
    st->set_ready(0);
    return future<T>(st);
}
template <typename T, typename E>
future<T> make_exceptional_future(E const& e) {
    return make_exceptional_future<T>(std::make_exception_ptr(e));
}

}  // namespace hpx
