// STREAM on one MI355X through the HIP backend's HPX C++ layer -- the shape
// of the reference's tests/performance/local/stream.cpp (run_benchmark
// :276-385, check_results :83-222): copy, scale, add, triad over
// hpx::compute::vector with par.on(default_executor), the benchmark's OWN
// functors (stream.cpp:224-271), and McCalpin's validation (eps 1e-13 for
// double).  Each functor is mapped to the device with a trait
// specialisation -- the only change a STREAM user makes.
//
// usage: stream_hip [--vector_size N] [--iterations K]
#include <hpx/hpx.hpp>
#include <hpx/hpx_init.hpp>
#include <hpx/util/lightweight_test.hpp>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <vector>

using STREAM_TYPE = double;

template <typename T>
struct multiply_step {
    explicit multiply_step(T factor) : factor_(factor) {}
    T operator()(T val) const { return val * factor_; }
    T factor_;
};
template <typename T>
struct add_step {
    T operator()(T val1, T val2) const { return val1 + val2; }
};
template <typename T>
struct triad_step {
    explicit triad_step(T factor) : factor_(factor) {}
    T operator()(T val1, T val2) const { return val1 + val2 * factor_; }
    T factor_;
};

namespace hpx { namespace compute { namespace hip { namespace traits {
template <typename T>
struct unary<::multiply_step<T>> {
    static constexpr int kind = HPXHIP_U_SCALE;
    template <typename C>
    static void scalars(::multiply_step<T> const& f, C* s) { s[0] = C(f.factor_); }
};
template <typename T>
struct binary<::add_step<T>> : detail::no_scalars<HPXHIP_B_ADD> {};
template <typename T>
struct binary<::triad_step<T>> {
    static constexpr int kind = HPXHIP_B_TRIAD;
    template <typename C>
    static void scalars(::triad_step<T> const& f, C* s) { s[0] = C(f.factor_); }
};
}}}}  // namespace hpx::compute::hip::traits

using Allocator = hpx::compute::hip::allocator<STREAM_TYPE>;
using Executor = hpx::compute::hip::default_executor;
using Vector = hpx::compute::vector<STREAM_TYPE, Allocator>;

static double mysecond() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// stream.cpp:83-222 restated: reproduce the recurrence, compare average
// relative error of each array against epsilon.
static bool check_results(std::size_t iterations, Vector const& a_res, Vector const& b_res, Vector const& c_res) {
    namespace ex = hpx::parallel::execution;
    std::vector<STREAM_TYPE> a(a_res.size()), b(b_res.size()), c(c_res.size());
    hpx::parallel::copy(ex::par, a_res.begin(), a_res.end(), a.begin());
    hpx::parallel::copy(ex::par, b_res.begin(), b_res.end(), b.begin());
    hpx::parallel::copy(ex::par, c_res.begin(), c_res.end(), c.begin());

    STREAM_TYPE aj = 1.0, bj = 2.0, cj = 0.0, scalar = 3.0;
    aj = 2.0E0 * aj;
    for (std::size_t k = 0; k < iterations; k++) {
        cj = aj;
        bj = scalar * cj;
        cj = aj + bj;
        aj = bj + scalar * cj;
    }
    STREAM_TYPE aSum = 0, bSum = 0, cSum = 0;
    for (std::size_t j = 0; j < a.size(); j++) {
        aSum += std::abs(a[j] - aj);
        bSum += std::abs(b[j] - bj);
        cSum += std::abs(c[j] - cj);
    }
    double const epsilon = sizeof(STREAM_TYPE) == 4 ? 1.e-6 : 1.e-13;
    double n = double(a.size());
    bool ok = std::abs(aSum / n / aj) <= epsilon && std::abs(bSum / n / bj) <= epsilon &&
              std::abs(cSum / n / cj) <= epsilon;
    if (ok) std::printf("Solution Validates: avg error less than %e on all three arrays\n", epsilon);
    else std::printf("Failed Validation: rel errors %e %e %e\n", aSum / n / aj, bSum / n / bj, cSum / n / cj);
    return ok;
}

int hpx_main(int argc, char* argv[]) {
    std::size_t vector_size = std::size_t(1) << 27, iterations = 10;
    for (int i = 1; i + 1 < argc; ++i) {
        if (!std::strcmp(argv[i], "--vector_size")) vector_size = std::strtoull(argv[i + 1], nullptr, 10);
        if (!std::strcmp(argv[i], "--iterations")) iterations = std::strtoull(argv[i + 1], nullptr, 10);
    }
    std::printf("Array size = %zu (elements), Memory per array = %.1f MiB\n", vector_size,
                sizeof(STREAM_TYPE) * (vector_size / 1024. / 1024.));
    std::printf("Each kernel will be executed %zu times.\n", iterations);

    hpx::compute::hip::target target;
    Allocator alloc(target);
    Vector a(vector_size, alloc), b(vector_size, alloc), c(vector_size, alloc);
    Executor exec(target);
    auto policy = hpx::parallel::execution::par.on(exec);

    hpx::parallel::fill(policy, a.begin(), a.end(), 1.0);
    hpx::parallel::fill(policy, b.begin(), b.end(), 2.0);
    hpx::parallel::fill(policy, c.begin(), c.end(), 0.0);
    hpx::parallel::transform(policy, a.begin(), a.end(), a.begin(), multiply_step<STREAM_TYPE>(2.0));

    std::vector<std::vector<double>> timing(4, std::vector<double>(iterations));
    double const scalar = 3.0;
    for (std::size_t it = 0; it != iterations; ++it) {
        timing[0][it] = mysecond();
        hpx::parallel::copy(policy, a.begin(), a.end(), c.begin());
        timing[0][it] = mysecond() - timing[0][it];

        timing[1][it] = mysecond();
        hpx::parallel::transform(policy, c.begin(), c.end(), b.begin(), multiply_step<STREAM_TYPE>(scalar));
        timing[1][it] = mysecond() - timing[1][it];

        timing[2][it] = mysecond();
        hpx::parallel::transform(policy, a.begin(), a.end(), b.begin(), b.end(), c.begin(), add_step<STREAM_TYPE>());
        timing[2][it] = mysecond() - timing[2][it];

        timing[3][it] = mysecond();
        hpx::parallel::transform(policy, b.begin(), b.end(), c.begin(), c.end(), a.begin(),
                                 triad_step<STREAM_TYPE>(scalar));
        timing[3][it] = mysecond() - timing[3][it];
    }
    bool ok = check_results(iterations, a, b, c);
    HPX_TEST(ok);

    char const* label[4] = {"Copy:      ", "Scale:     ", "Add:       ", "Triad:     "};
    double const bytes[4] = {2. * sizeof(STREAM_TYPE) * vector_size, 2. * sizeof(STREAM_TYPE) * vector_size,
                             3. * sizeof(STREAM_TYPE) * vector_size, 3. * sizeof(STREAM_TYPE) * vector_size};
    std::printf("Function    Best Rate MB/s  Avg time     Min time     Max time\n");
    for (int j = 0; j < 4; ++j) {
        double mn = 1e30, mx = 0, avg = 0;
        for (std::size_t k = 1; k < iterations; ++k) {  // first iteration excluded (stream.cpp:489)
            mn = std::min(mn, timing[j][k]);
            mx = std::max(mx, timing[j][k]);
            avg += timing[j][k];
        }
        avg /= double(iterations > 1 ? iterations - 1 : 1);
        std::printf("%s%12.1f  %11.6f  %11.6f  %11.6f\n", label[j], 1.0E-06 * bytes[j] / mn, avg, mn, mx);
    }
    return hpx::finalize();
}

int main(int argc, char* argv[]) {
    HPX_TEST_EQ(hpx::init(argc, argv), 0);
    int errors = hpx::util::report_errors();
    if (!errors) std::cout << "stream_hip: all tests passed" << std::endl;
    return errors;
}
