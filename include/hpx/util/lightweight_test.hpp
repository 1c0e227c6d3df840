// hpx/util/lightweight_test.hpp -- the HPX_TEST* assertion macros used by the
// reference's unit tests (hpx/util/lightweight_test.hpp in HPX 1.4.0): a
// failed check prints file:line and is counted; report_errors() returns the
// count as the process exit status.
#pragma once

#include <atomic>
#include <iostream>

namespace hpx { namespace util { namespace detail {
inline std::atomic<int>& error_count() {
    static std::atomic<int> n{0};
    return n;
}
// Each operand is evaluated exactly once (an operand may be a call with side
// effects, e.g. HPX_TEST_EQ(hpx::init(argc, argv), 0)).
template <typename A, typename B, typename Rel>
bool check_rel(A const& a, B const& b, Rel rel, char const* expr, char const* file, int line) {
    bool ok = rel(a, b);
    if (!ok) {
        ++error_count();
        std::cerr << file << "(" << line << "): test '" << expr << "' failed (" << a << " vs " << b << ")\n";
    }
    return ok;
}
}  // namespace detail

inline int report_errors() {
    int n = detail::error_count().load();
    if (n) std::cerr << n << " error(s) detected.\n";
    return n;
}
}}  // namespace hpx::util

#define HPX_TEST(expr)                                                                          \
    ((expr) ? true                                                                              \
            : (++::hpx::util::detail::error_count(),                                            \
               (std::cerr << __FILE__ << "(" << __LINE__ << "): test '" #expr "' failed\n"), false))
#define HPX_TEST_MSG(expr, msg)                                                                 \
    ((expr) ? true                                                                              \
            : (++::hpx::util::detail::error_count(),                                            \
               (std::cerr << __FILE__ << "(" << __LINE__ << "): " << (msg) << "\n"), false))
#define HPX_TEST_REL_(a, b, OP)                                                                   \
    ::hpx::util::detail::check_rel(                                                               \
        (a), (b), [](auto const& x_, auto const& y_) { return bool(x_ OP y_); }, #a " " #OP " " #b, \
        __FILE__, __LINE__)
#define HPX_TEST_EQ(a, b) HPX_TEST_REL_(a, b, ==)
#define HPX_TEST_NEQ(a, b) HPX_TEST_REL_(a, b, !=)
#define HPX_TEST_LT(a, b) HPX_TEST_REL_(a, b, <)
#define HPX_TEST_LTE(a, b) HPX_TEST_REL_(a, b, <=)
#define HPX_TEST_EQ_MSG(a, b, msg) HPX_TEST_MSG((a) == (b), msg)
