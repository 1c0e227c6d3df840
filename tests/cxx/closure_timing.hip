// Timing of the arbitrary-callable (device closure) paths against the
// built-in operator kinds at benchmark scale:
//
//   transform_reduce  2^30 int64 / f64: std::plus + identity (kind path,
//                     libhpxhip) vs a lambda conv (built-in red) vs a lambda
//                     red + lambda conv (red lifted to opt<T>)
//                     transform_reduce.hpp:254
//   inclusive_scan    2^30 int64 / f64: std::plus vs a lambda op (lifted)
//                     inclusive_scan.hpp:288-606
//   copy_if           2^30 int64, 50 % selected: not_less_than<0> vs a lambda
//                     copy.hpp:585
//   sort              2^28 u64: radix sort (std::less) vs a lambda comparator
//                     (merge sort), sort.hpp:364
//
// Device time per call from HIP events on the policy's stream, best of 5
// after one warm-up; GB/s on the algorithmic bytes (8 B/elem reduce, 16 B/elem
// scan, 12 B/elem copy_if at 50 %).  Each result is also checked against the
// kind path's.  usage: closure_timing [logn=30] [reduce|sort|all]
#include <hpx/hpx.hpp>
#include <hpx/hpx_init.hpp>
#include <hpx/util/lightweight_test.hpp>

#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>

namespace hip = hpx::compute::hip;
namespace ex = hpx::parallel::execution;
namespace fn = hpx::compute::hip::functional;
template <typename T>
using dvec = hpx::compute::vector<T, hip::allocator<T>>;

struct timer {
    hpxhip_event a = nullptr, b = nullptr;
    hpxhip_stream s;
    explicit timer(hpxhip_stream st) : s(st) {
        hpxhip_event_create(&a);
        hpxhip_event_create(&b);
    }
    ~timer() {
        hpxhip_event_destroy(a);
        hpxhip_event_destroy(b);
    }
    template <typename F>
    double best_ms(F&& f, int reps = 5) {
        f();
        double best = 1e30;
        for (int r = 0; r < reps; ++r) {
            hpxhip_event_record(a, s);
            f();
            hpxhip_event_record(b, s);
            hpxhip_event_synchronize(b);
            float ms = 0;
            hpxhip_event_elapsed_ms(a, b, &ms);
            best = ms < best ? ms : best;
        }
        return best;
    }
};

void row(char const* what, std::size_t n, double bytes_per_elem, double ms, double ref_ms) {
    const double gbs = bytes_per_elem * double(n) / (ms * 1e-3) / 1e9;
    std::printf("%-52s %10.4f ms %9.1f GB/s %6.1f %% HBM  x%.3f of the kind path\n", what, ms, gbs, gbs / 80.0,
                ms / ref_ms);
    std::fflush(stdout);
}

template <typename T>
void reductions(hip::default_executor& exec, std::size_t n, char const* tn) {
    auto pol = ex::par.on(exec);
    dvec<T> d(n, hip::allocator<T>(exec.target()));
    // integers in [-2^20, 2^20] (exact sums), doubles in [0, 1)
    if constexpr (std::is_integral<T>::value)
        hip::detail::check(hpxhip_generate(hip::dtype_of<T>::value, HPXHIP_GEN_RANGE, 0x5eed, -(1 << 20), 1 << 20,
                                           d.data(), n, exec.target().stream()), "generate");
    else
        hip::detail::check(hpxhip_generate(hip::dtype_of<T>::value, HPXHIP_GEN_UNIT, 0x5eed, 0, 0, d.data(), n,
                                           exec.target().stream()), "generate");
    // the policy holds a copy of exec, whose target has a stream of its own
    // (cuda_target.cpp:203-211): time on that stream, after the generate
    exec.target().synchronize();
    timer tm(pol.executor().target().stream());
    T kind_v{}, l1{}, l2{};
    double kind = tm.best_ms([&] { kind_v = hpx::parallel::transform_reduce(pol, d.begin(), d.end(), T(0), std::plus<T>(), fn::identity{}); });
    double conv = tm.best_ms([&] {
        l1 = hpx::parallel::transform_reduce(pol, d.begin(), d.end(), T(0), std::plus<T>(), [] HPX_HOST_DEVICE(T x) { return x; });
    });
    double lifted = tm.best_ms([&] {
        l2 = hpx::parallel::transform_reduce(pol, d.begin(), d.end(), T(0), [] HPX_HOST_DEVICE(T a, T b) { return a + b; },
                                             [] HPX_HOST_DEVICE(T x) { return x; });
    });
    std::string base = std::string("transform_reduce ") + tn;
    row((base + " std::plus + identity (kind)").c_str(), n, 8, kind, kind);
    row((base + " std::plus + lambda conv").c_str(), n, 8, conv, kind);
    row((base + " lambda red + lambda conv (lifted)").c_str(), n, 8, lifted, kind);
    if constexpr (std::is_integral<T>::value) {
        HPX_TEST_EQ(l1, kind_v);
        HPX_TEST_EQ(l2, kind_v);
    }

    dvec<T> o(n, hip::allocator<T>(exec.target()));
    double skind = tm.best_ms([&] { hpx::parallel::inclusive_scan(pol, d.begin(), d.end(), o.begin(), std::plus<T>(), T(0)); });
    T last_kind = o[n - 1];
    double slam = tm.best_ms([&] {
        hpx::parallel::inclusive_scan(pol, d.begin(), d.end(), o.begin(), [] HPX_HOST_DEVICE(T a, T b) { return a + b; }, T(0));
    });
    base = std::string("inclusive_scan ") + tn;
    row((base + " std::plus (kind)").c_str(), n, 16, skind, skind);
    row((base + " lambda op (lifted)").c_str(), n, 16, slam, skind);
    if constexpr (std::is_integral<T>::value) HPX_TEST_EQ(T(o[n - 1]), last_kind);

    if constexpr (std::is_integral<T>::value) {
        std::size_t ck = 0, cl = 0;
        double ckind = tm.best_ms([&] {
            ck = std::size_t(hpx::parallel::copy_if(pol, d.begin(), d.end(), o.begin(), fn::not_less_than<T>{0}).out() - o.begin());
        });
        double clam = tm.best_ms([&] {
            cl = std::size_t(hpx::parallel::copy_if(pol, d.begin(), d.end(), o.begin(), [] HPX_HOST_DEVICE(T x) { return !(x < 0); }).out() -
                             o.begin());
        });
        base = std::string("copy_if ") + tn;
        row((base + " not_less_than<0> (kind)").c_str(), n, 12, ckind, ckind);
        row((base + " lambda pred").c_str(), n, 12, clam, ckind);
        HPX_TEST_EQ(ck, cl);
    }
}

void sorts(hip::default_executor& exec, std::size_t n) {
    auto pol = ex::par.on(exec);
    dvec<uint64_t> d(n, hip::allocator<uint64_t>(exec.target()));
    // keys generated and sorted on the policy's stream (a copy of exec has a
    // stream of its own: generating on exec's would race the sort)
    const hpxhip_stream ps = pol.executor().target().stream();
    timer tm(ps);
    auto regen = [&] {
        hip::detail::check(hpxhip_generate(HPXHIP_U64, HPXHIP_GEN_BITS, 0xabc, 0, 0, d.data(), n, ps), "generate");
    };
    double gen = tm.best_ms(regen);
    double radix = tm.best_ms([&] {
        regen();
        hpx::parallel::sort(pol, d.begin(), d.end());
    }) - gen;
    std::printf("%-52s %10.4f ms %9.2f Gkeys/s\n", "sort u64 std::less (radix)", radix, double(n) / radix / 1e6);
    std::fflush(stdout);
    double merge = tm.best_ms([&] {
        regen();
        hpx::parallel::sort(pol, d.begin(), d.end(), [] HPX_HOST_DEVICE(uint64_t a, uint64_t b) { return a < b; });
    }, 3) - gen;
    HPX_TEST(hpx::parallel::is_sorted(pol, d.begin(), d.end()));
    std::printf("%-52s %10.4f ms %9.2f Gkeys/s  x%.2f of the radix sort\n", "sort u64 lambda comparator (merge sort)",
                merge, double(n) / merge / 1e6, merge / radix);
}

int hpx_main(int argc, char* argv[]) {
    const int logn = argc > 1 ? std::atoi(argv[1]) : 30;
    const std::string what = argc > 2 ? argv[2] : "all";
    hip::target t;
    hip::default_executor exec(t);
    std::printf("closure paths vs the built-in kinds, n = 2^%d (sort: 2^%d)\n", logn, logn - 2);
    if (what != "sort") {
        reductions<int64_t>(exec, std::size_t(1) << logn, "int64");
        reductions<double>(exec, std::size_t(1) << logn, "f64");
    }
    if (what != "reduce") sorts(exec, std::size_t(1) << (logn - 2));
    return hpx::finalize();
}

int main(int argc, char* argv[]) {
    HPX_TEST_EQ(hpx::init(argc, argv), 0);
    int errors = hpx::util::report_errors();
    if (!errors) std::printf("closure_timing: all tests passed\n");
    return errors;
}
