// hpx/compute/hip/functional.hpp -- the element functors the HIP backend runs,
// and the traits that map a C++ function object onto a device kernel.
//
// The reference instantiates a device kernel per user closure
// (hpx/compute/cuda/detail/launch.hpp:32-137); a C ABI cannot take closures,
// so each algorithm maps its function object through a trait to one of the
// library's built-in element operations (include/hpxhip.h enums):
//
//   traits::unary<F>   -> HPXHIP_U_*   (for_each, transform, transform_reduce
//                                       and transform_*_scan conversions)
//   traits::binary<F>  -> HPXHIP_B_*   (binary transform, inner products)
//   traits::binop<F>   -> HPXHIP_*     (reduce / scan operators)
//   traits::pred<F>    -> HPXHIP_P_*   (copy_if)
//   traits::compare<F> -> ascending / descending (sort, sort_by_key)
//
// A user functor with the same meaning as a built-in one opts in by
// specialising the trait, e.g. the STREAM benchmark's own
// `multiply_step<T>` (tests/cxx/stream_hip.cpp):
//
//   template <typename T>
//   struct hpx::compute::hip::traits::unary<multiply_step<T>> {
//       static constexpr int kind = HPXHIP_U_SCALE;
//       template <typename C> static void scalars(multiply_step<T> const& f, C* s)
//       { s[0] = f.factor_; }
//   };
//
// Using a function object with no trait is a compile-time error that names
// the trait to specialise -- never a silent host fallback.
#pragma once

#include <hpx/config/compiler_specific.hpp>
#include <hpxhip.h>

#include <functional>
#include <tuple>
#include <type_traits>

namespace hpx { namespace compute { namespace hip {

namespace functional {
// ---- unary element functors (also callable on the host) -----------------
struct identity {
    template <typename T> HPX_HOST_DEVICE T operator()(T x) const { return x; }
};
template <typename T>
struct multiply_step {  // stream.cpp:224-237
    using compute_type = T;
    T factor;
    HPX_HOST_DEVICE T operator()(T x) const { return x * factor; }
};
template <typename T>
struct add_value {  // for_each_compute.cu:40 `i += 5`
    using compute_type = T;
    T value;
    HPX_HOST_DEVICE T operator()(T x) const { return x + value; }
};
template <typename T>
struct affine {
    using compute_type = T;
    T a, b;
    HPX_HOST_DEVICE T operator()(T x) const { return x * a + b; }
};
struct negate {
    template <typename T> HPX_HOST_DEVICE T operator()(T x) const { return -x; }
};
struct absolute {
    template <typename T> HPX_HOST_DEVICE T operator()(T x) const { return x < T(0) ? -x : x; }
};
struct square {
    template <typename T> HPX_HOST_DEVICE T operator()(T x) const { return x * x; }
};

// ---- binary element functors ---------------------------------------------
struct add_step {  // stream.cpp:240-253
    template <typename T> HPX_HOST_DEVICE T operator()(T x, T y) const { return x + y; }
};
template <typename T>
struct triad_step {  // stream.cpp:256-271, transform_compute.cu:36
    using compute_type = T;
    T factor;
    HPX_HOST_DEVICE T operator()(T x, T y) const { return x + y * factor; }
};
struct subtract {
    template <typename T> HPX_HOST_DEVICE T operator()(T x, T y) const { return x - y; }
};
struct multiply {
    template <typename T> HPX_HOST_DEVICE T operator()(T x, T y) const { return x * y; }
};
template <typename T>
struct axpy {
    using compute_type = T;
    T a;
    HPX_HOST_DEVICE T operator()(T x, T y) const { return x * a + y; }
};

// ---- for_loop bodies ----------------------------------------------------------
// for_loop_n(policy, first, n, induction(b), induction(c), body) passes the
// body one iterator per loop variable (position 0 = the loop iterator, then
// the inductions in call order).  loop_assign<Out, F, In...> is the body
// `*v[Out] = f(*v[In]...)`; for_loop_compute.cu:40-48's lambda
// `*C = *A + 3.0 * *B` is loop_assign<2, triad_step<double>, 0, 1>{{3.0}}.
template <std::size_t Out, typename F, std::size_t... In>
struct loop_assign {
    static_assert(sizeof...(In) == 1 || sizeof...(In) == 2, "loop_assign: one or two inputs");
    F f;
    template <typename... P>
    void operator()(P... p) const {  // host meaning (pointers / iterators)
        auto t = std::make_tuple(p...);
        *std::get<Out>(t) = f(*std::get<In>(t)...);
    }
};

// loop_accumulate<Red, F, In...> is the body of a for_loop with a reduction:
// `r = op(r, f(*v[In]...))` where r is the reduction at position Red;
// for_loop_reduction.cpp:37-44's `[](iterator it, std::size_t& sum) { sum +=
// *it; }` is loop_accumulate<1, identity, 0>{}.
template <std::size_t Red, typename F, std::size_t... In>
struct loop_accumulate {
    static_assert(sizeof...(In) == 1 || sizeof...(In) == 2, "loop_accumulate: one or two inputs");
    static constexpr std::size_t red = Red;
    F f;
};

// loop_accumulate_all<A...> is the body of a for_loop with several
// reductions (for_loop.hpp:802-812 takes any number): one loop_accumulate per
// reduction, e.g. `[](it, T& sum, T& sq) { sum += *it; sq += *it * *it; }` is
// accumulate_all(loop_accumulate<1, identity>{}, loop_accumulate<2, square>{})
// (template arguments of the inputs omitted).  Up to eight reductions (their
// views travel back in one 64-byte result slot).
template <typename... A>
struct loop_accumulate_all {
    static_assert(sizeof...(A) >= 1 && sizeof...(A) <= 8, "loop_accumulate_all: one to eight reductions");
    std::tuple<A...> parts;
};
template <typename... A>
loop_accumulate_all<A...> accumulate_all(A const&... a) {
    return {std::tuple<A...>(a...)};
}

// ---- reduction operators not in <functional> ------------------------------
struct minimum {
    template <typename T> HPX_HOST_DEVICE T operator()(T x, T y) const { return y < x ? y : x; }
};
struct maximum {
    template <typename T> HPX_HOST_DEVICE T operator()(T x, T y) const { return x < y ? y : x; }
};

// ---- predicates -------------------------------------------------------------
#define HPXHIP_PREDICATE(NAME, EXPR)                                  \
    template <typename T>                                             \
    struct NAME {                                                     \
        T value;                                                      \
        HPX_HOST_DEVICE bool operator()(T x) const { return EXPR; }   \
    };
HPXHIP_PREDICATE(less_than, x < value)
HPXHIP_PREDICATE(less_equal, x <= value)
HPXHIP_PREDICATE(greater_than, x > value)
HPXHIP_PREDICATE(greater_equal, x >= value)
HPXHIP_PREDICATE(equal_to, x == value)
HPXHIP_PREDICATE(not_equal_to, x != value)
HPXHIP_PREDICATE(not_less_than, !(x < value))  // copyif_random.cpp:45
HPXHIP_PREDICATE(any_bits, (x & value) != 0)
#undef HPXHIP_PREDICATE
}  // namespace functional

namespace traits {
// Primary templates are declared, not defined: an unmapped functor fails to
// compile at the use site with "incomplete type traits::unary<F>".
template <typename F, typename Enable = void> struct unary;
template <typename F, typename Enable = void> struct binary;
template <typename F, typename Enable = void> struct binop;
template <typename F, typename Enable = void> struct pred;
template <typename F, typename Enable = void> struct compare;

namespace detail {
template <int K>
struct no_scalars {
    static constexpr int kind = K;
    template <typename F, typename C> static void scalars(F const&, C*) {}
};
template <typename T, typename = void>
struct is_complete : std::false_type {};
template <typename T>
struct is_complete<T, decltype(void(sizeof(T)))> : std::true_type {};
}  // namespace detail

template <> struct unary<functional::identity> : detail::no_scalars<HPXHIP_U_IDENTITY> {};
template <> struct unary<functional::negate> : detail::no_scalars<HPXHIP_U_NEGATE> {};
template <> struct unary<functional::absolute> : detail::no_scalars<HPXHIP_U_ABS> {};
template <> struct unary<functional::square> : detail::no_scalars<HPXHIP_U_SQUARE> {};
template <typename T> struct unary<functional::multiply_step<T>> {
    static constexpr int kind = HPXHIP_U_SCALE;
    template <typename C> static void scalars(functional::multiply_step<T> const& f, C* s) { s[0] = C(f.factor); }
};
template <typename T> struct unary<functional::add_value<T>> {
    static constexpr int kind = HPXHIP_U_ADD_SCALAR;
    template <typename C> static void scalars(functional::add_value<T> const& f, C* s) { s[0] = C(f.value); }
};
template <typename T> struct unary<functional::affine<T>> {
    static constexpr int kind = HPXHIP_U_AFFINE;
    template <typename C> static void scalars(functional::affine<T> const& f, C* s) {
        s[0] = C(f.a);
        s[1] = C(f.b);
    }
};
template <typename T> struct unary<std::negate<T>> : detail::no_scalars<HPXHIP_U_NEGATE> {};

template <> struct binary<functional::add_step> : detail::no_scalars<HPXHIP_B_ADD> {};
template <> struct binary<functional::subtract> : detail::no_scalars<HPXHIP_B_SUB> {};
template <> struct binary<functional::multiply> : detail::no_scalars<HPXHIP_B_MUL> {};
template <> struct binary<functional::minimum> : detail::no_scalars<HPXHIP_B_MIN> {};
template <> struct binary<functional::maximum> : detail::no_scalars<HPXHIP_B_MAX> {};
template <typename T> struct binary<std::plus<T>> : detail::no_scalars<HPXHIP_B_ADD> {};
template <typename T> struct binary<std::minus<T>> : detail::no_scalars<HPXHIP_B_SUB> {};
template <typename T> struct binary<std::multiplies<T>> : detail::no_scalars<HPXHIP_B_MUL> {};
template <typename T> struct binary<functional::triad_step<T>> {
    static constexpr int kind = HPXHIP_B_TRIAD;
    template <typename C> static void scalars(functional::triad_step<T> const& f, C* s) { s[0] = C(f.factor); }
};
template <typename T> struct binary<functional::axpy<T>> {
    static constexpr int kind = HPXHIP_B_AXPY;
    template <typename C> static void scalars(functional::axpy<T> const& f, C* s) { s[0] = C(f.a); }
};

template <typename T> struct binop<std::plus<T>> : detail::no_scalars<HPXHIP_PLUS> {};
template <typename T> struct binop<std::multiplies<T>> : detail::no_scalars<HPXHIP_MULTIPLIES> {};
template <typename T> struct binop<std::bit_and<T>> : detail::no_scalars<HPXHIP_BIT_AND> {};
template <typename T> struct binop<std::bit_or<T>> : detail::no_scalars<HPXHIP_BIT_OR> {};
template <typename T> struct binop<std::bit_xor<T>> : detail::no_scalars<HPXHIP_BIT_XOR> {};
template <> struct binop<functional::add_step> : detail::no_scalars<HPXHIP_PLUS> {};
template <> struct binop<functional::multiply> : detail::no_scalars<HPXHIP_MULTIPLIES> {};
template <> struct binop<functional::minimum> : detail::no_scalars<HPXHIP_MIN> {};
template <> struct binop<functional::maximum> : detail::no_scalars<HPXHIP_MAX> {};

#define HPXHIP_PRED_TRAIT(NAME, KIND)                                               \
    template <typename T> struct pred<functional::NAME<T>> {                        \
        static constexpr int kind = KIND;                                           \
        static T arg(functional::NAME<T> const& f) { return f.value; }              \
    };
HPXHIP_PRED_TRAIT(less_than, HPXHIP_P_LT)
HPXHIP_PRED_TRAIT(less_equal, HPXHIP_P_LE)
HPXHIP_PRED_TRAIT(greater_than, HPXHIP_P_GT)
HPXHIP_PRED_TRAIT(greater_equal, HPXHIP_P_GE)
HPXHIP_PRED_TRAIT(equal_to, HPXHIP_P_EQ)
HPXHIP_PRED_TRAIT(not_equal_to, HPXHIP_P_NE)
HPXHIP_PRED_TRAIT(not_less_than, HPXHIP_P_NOT_LT)
HPXHIP_PRED_TRAIT(any_bits, HPXHIP_P_BITS)
#undef HPXHIP_PRED_TRAIT

template <typename T> struct compare<std::less<T>> { static constexpr bool descending = false; };
template <typename T> struct compare<std::greater<T>> { static constexpr bool descending = true; };

template <typename F> using unary_t = unary<typename std::decay<F>::type>;
template <typename F> using binary_t = binary<typename std::decay<F>::type>;
template <typename F> using binop_t = binop<typename std::decay<F>::type>;
template <typename F> using pred_t = pred<typename std::decay<F>::type>;
template <typename F> using compare_t = compare<typename std::decay<F>::type>;

// Arithmetic type of a transform: the trait's compute_type, else the
// functor's (triad_step<double> over int vectors computes in double,
// transform_compute.cu:36), else the element type.
namespace detail {
template <typename F, typename E, typename = void>
struct functor_compute { using type = E; };
template <typename F, typename E>
struct functor_compute<F, E, std::void_t<typename F::compute_type>> { using type = typename F::compute_type; };
}  // namespace detail
template <typename Tr, typename F, typename E, typename = void>
struct compute_of { using type = typename detail::functor_compute<F, E>::type; };
template <typename Tr, typename F, typename E>
struct compute_of<Tr, F, E, std::void_t<typename Tr::compute_type>> { using type = typename Tr::compute_type; };
template <typename Tr, typename F, typename E>
using compute_t = typename compute_of<Tr, typename std::decay<F>::type, E>::type;

template <typename F> constexpr bool is_binop = detail::is_complete<binop_t<F>>::value;
template <typename F> constexpr bool is_unary = detail::is_complete<unary_t<F>>::value;
}  // namespace traits
}}}  // namespace hpx::compute::hip
