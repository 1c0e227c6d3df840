// hpx/parallel/execution.hpp -- execution policies of HPX 1.4.0 as the HIP
// backend sees them.
//
//   seq, par, par_unseq, task      <- hpx/parallel/execution_policy.hpp:60-1030
//   policy.on(executor)            <- execution_policy.hpp:140-160 (rebind_executor)
//   policy.with(parameters...)     <- execution_policy.hpp:175-195
//   static_chunk_size & friends    <- hpx/parallel/executors/static_chunk_size.hpp
//   algorithm_result<Policy, T>    <- hpx/parallel/util/detail/algorithm_result.hpp:20-160
//                                     (T for synchronous policies, future<T> for task)
//
// Chunking parameters are accepted for source compatibility and ignored: the
// device kernels choose their own tiling (DESIGN.md "Kernels").
#pragma once

#include <hpx/compute/hip.hpp>
#include <hpx/config/compiler_specific.hpp>

#include <cstddef>
#include <type_traits>

namespace hpx { namespace parallel { namespace execution {

struct task_policy_tag {};
constexpr task_policy_tag task{};

struct sequenced_execution_tag {};
struct parallel_execution_tag {};

struct no_executor {};

template <typename Category, bool Task, typename Executor = no_executor>
class policy {
    Executor exec_{};

public:
    using execution_category = Category;
    using executor_type = Executor;
    static constexpr bool is_task = Task;
    static constexpr bool has_executor = !std::is_same<Executor, no_executor>::value;

    constexpr policy() = default;
    explicit policy(Executor const& e) : exec_(e) {}

    policy<Category, true, Executor> operator()(task_policy_tag) const {
        if constexpr (has_executor) return policy<Category, true, Executor>(exec_);
        else return policy<Category, true, Executor>();
    }
    template <typename E>
    policy<Category, Task, E> on(E const& e) const {
        return policy<Category, Task, E>(e);
    }
    template <typename... Params>
    policy const& with(Params&&...) const {
        return *this;
    }
    Executor const& executor() const { return exec_; }
};

using sequenced_policy = policy<sequenced_execution_tag, false>;
using sequenced_task_policy = policy<sequenced_execution_tag, true>;
using parallel_policy = policy<parallel_execution_tag, false>;
using parallel_task_policy = policy<parallel_execution_tag, true>;
struct parallel_unsequenced_policy : policy<parallel_execution_tag, false> {};

constexpr sequenced_policy seq{};
constexpr parallel_policy par{};
constexpr parallel_unsequenced_policy par_unseq{};

template <typename T>
struct is_execution_policy : std::false_type {};
template <typename C, bool Task, typename E>
struct is_execution_policy<policy<C, Task, E>> : std::true_type {};
template <>
struct is_execution_policy<parallel_unsequenced_policy> : std::true_type {};

template <typename T>
struct is_async_execution_policy : std::false_type {};
template <typename C, typename E>
struct is_async_execution_policy<policy<C, true, E>> : std::true_type {};

// ------------------------------------------------------- executor concept
// Traits (hpx/traits/is_executor.hpp, executor_traits.hpp); an executor
// opts in by specialisation, as default_executor.hpp:233-260 does.
template <typename Executor, typename Enable = void>
struct executor_execution_category {
    using type = parallel_execution_tag;
};
template <typename T> struct is_one_way_executor : std::false_type {};
template <typename T> struct is_two_way_executor : std::false_type {};
template <typename T> struct is_bulk_one_way_executor : std::false_type {};
template <typename T> struct is_bulk_two_way_executor : std::false_type {};
template <typename T>
struct is_executor_any
  : std::integral_constant<bool, is_one_way_executor<T>::value || is_two_way_executor<T>::value ||
                                     is_bulk_one_way_executor<T>::value || is_bulk_two_way_executor<T>::value> {};

// Customisation points (executors/execution.hpp:650-795): forward to the
// executor's members.
template <typename Executor, typename F, typename... Ts>
void post(Executor&& exec, F&& f, Ts&&... ts) {
    exec.post(std::forward<F>(f), std::forward<Ts>(ts)...);
}
template <typename Executor, typename F, typename... Ts>
auto async_execute(Executor&& exec, F&& f, Ts&&... ts) {
    return exec.async_execute(std::forward<F>(f), std::forward<Ts>(ts)...);
}
template <typename Executor, typename F, typename... Ts>
void sync_execute(Executor&& exec, F&& f, Ts&&... ts) {
    exec.sync_execute(std::forward<F>(f), std::forward<Ts>(ts)...);
}
template <typename Executor, typename F, typename Shape, typename... Ts>
auto bulk_async_execute(Executor&& exec, F&& f, Shape const& shape, Ts&&... ts) {
    return exec.bulk_async_execute(std::forward<F>(f), shape, std::forward<Ts>(ts)...);
}
template <typename Executor, typename F, typename Shape, typename... Ts>
void bulk_sync_execute(Executor&& exec, F&& f, Shape const& shape, Ts&&... ts) {
    exec.bulk_sync_execute(std::forward<F>(f), shape, std::forward<Ts>(ts)...);
}

// executor parameters (accepted, ignored)
struct static_chunk_size {
    std::size_t chunk = 0;
    static_chunk_size() = default;
    explicit static_chunk_size(std::size_t c) : chunk(c) {}
};
struct dynamic_chunk_size {
    std::size_t chunk = 1;
    explicit dynamic_chunk_size(std::size_t c = 1) : chunk(c) {}
};
struct guided_chunk_size {
    std::size_t chunk = 1;
    explicit guided_chunk_size(std::size_t c = 1) : chunk(c) {}
};
struct auto_chunk_size {};

}  // namespace execution

namespace util { namespace detail {
template <typename Policy, typename T = void>
struct algorithm_result {
    using type = typename std::conditional<
        execution::is_async_execution_policy<typename std::decay<Policy>::type>::value, hpx::future<T>, T>::type;
};
}}  // namespace util::detail

// hpx::util::tagged_pair / tagged_tuple results of copy, transform, copy_if,
// sort_by_key (hpx/util/tagged_pair.hpp); accessors named by the tags.
namespace util {
// hpx/parallel/util/projection_identity.hpp: the default projection of the
// algorithms that take one (sort.hpp:364).
struct projection_identity {
    template <typename T>
    HPX_HOST_DEVICE constexpr T operator()(T v) const {
        return v;
    }
};

template <typename A, typename B>
struct tagged_pair {
    A first;
    B second;
    A in() const { return first; }
    B out() const { return second; }
    A in1() const { return first; }
    B in2() const { return second; }
};
template <typename A, typename B, typename C>
struct tagged_tuple {
    A first;
    B second;
    C third;
    A in1() const { return first; }
    B in2() const { return second; }
    C out() const { return third; }
};
}  // namespace util
}}  // namespace hpx::parallel

namespace hpx { namespace util {
template <std::size_t I, typename A, typename B>
auto get(parallel::util::tagged_pair<A, B> const& p) {
    if constexpr (I == 0) return p.first;
    else return p.second;
}
template <std::size_t I, typename A, typename B, typename C>
auto get(parallel::util::tagged_tuple<A, B, C> const& p) {
    if constexpr (I == 0) return p.first;
    else if constexpr (I == 1) return p.second;
    else return p.third;
}
}}  // namespace hpx::util
