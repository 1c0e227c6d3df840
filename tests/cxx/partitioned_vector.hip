// hpx::partitioned_vector over HIP targets and its segmented algorithms,
// compiled by hipcc (device closures as in the reference's example):
//   examples/compute/cuda/partitioned_vector.cu:27-53   for_each(pfo) under seq, par,
//                                                        seq(task), par(task)
//   tests/unit/parallel/segmented_algorithms/partitioned_vector_reduce.cpp:26-76
//                                                        10007 ones, init 1 -> 10008 (int, double)
//   partitioned_vector_inclusive_scan.cpp:225-340        iota from 1 vs sequential_inclusive_scan,
//                                                        layouts: one per target, (3), (1000);
//                                                        in place; exclusive too
// plus transform, copy to/from the host, and a segment-order FP reduce.
#include <hpx/hpx.hpp>
#include <hpx/hpx_init.hpp>
#include <hpx/include/partitioned_vector.hpp>
#include <hpx/util/lightweight_test.hpp>

#include <cstdint>
#include <iostream>
#include <numeric>
#include <vector>

namespace hip = hpx::compute::hip;
namespace ex = hpx::parallel::execution;
namespace fn = hpx::compute::hip::functional;

template <typename T>
using pvec = hpx::partitioned_vector<T, hpx::compute::vector<T, hip::allocator<T>>>;

template <typename T>
std::vector<T> to_host(pvec<T> const& v) {
    std::vector<T> h(v.size());
    hpx::parallel::copy(ex::par, v.begin(), v.end(), h.begin());
    return h;
}

// partitioned_vector.cu:27-35
struct pfo {
    template <typename T>
    HPX_HOST_DEVICE void operator()(T& val) const {
        int v = val;
        val = ++v;
    }
};

void test_example(hip::target_distribution_policy const& policy) {
    pvec<int> v(1000, policy);
    hpx::parallel::for_each(ex::seq, v.begin(), v.end(), pfo());
    hpx::parallel::for_each(ex::par, v.begin(), v.end(), pfo());
    hpx::parallel::for_each(ex::seq(ex::task), v.begin(), v.end(), pfo()).get();
    hpx::parallel::for_each(ex::par(ex::task), v.begin(), v.end(), pfo()).get();
    std::vector<int> h = to_host(v);
    for (std::size_t i = 0; i != h.size(); ++i)
        if (!HPX_TEST_EQ(h[i], 4)) break;
}

// partitioned_vector_reduce.cpp:26-76
template <typename T>
void test_reduce(hip::target_distribution_policy const& policy) {
    std::size_t const num = 10007;
    pvec<T> const xvalues(num, T(1), policy);
    HPX_TEST_EQ(hpx::parallel::reduce(ex::seq, xvalues.begin(), xvalues.end(), T(1), std::plus<T>()), T(num + 1));
    HPX_TEST_EQ(hpx::parallel::reduce(ex::par, xvalues.begin(), xvalues.end(), T(1), std::plus<T>()), T(num + 1));
    HPX_TEST_EQ(hpx::parallel::reduce(ex::seq(ex::task), xvalues.begin(), xvalues.end(), T(1), std::plus<T>()).get(),
                T(num + 1));
    HPX_TEST_EQ(hpx::parallel::reduce(ex::par(ex::task), xvalues.begin(), xvalues.end(), T(1), std::plus<T>()).get(),
                T(num + 1));
}

// partitioned_vector_inclusive_scan.cpp:225-340 (and the exclusive twin)
template <typename T>
void test_scans(std::size_t size, hip::target_distribution_policy const& policy) {
    pvec<T> in(size, policy);
    std::vector<T> h(size);
    std::iota(h.begin(), h.end(), T(1));
    hpx::parallel::copy(ex::par, h.begin(), h.end(), in.begin());
    std::vector<T> ver(size);
    std::partial_sum(h.begin(), h.end(), ver.begin());

    pvec<T> out(size, policy);
    hpx::parallel::inclusive_scan(ex::seq, in.begin(), in.end(), out.begin(), std::plus<T>(), T(0));
    HPX_TEST(to_host(out) == ver);
    hpx::parallel::fill(ex::par, out.begin(), out.end(), T(0));
    hpx::parallel::inclusive_scan(ex::par(ex::task), in.begin(), in.end(), out.begin(), std::plus<T>(), T(0)).get();
    HPX_TEST(to_host(out) == ver);

    std::vector<T> xver(size);
    T acc = T(50);
    for (std::size_t i = 0; i < size; ++i) {
        xver[i] = acc;
        acc += h[i];
    }
    hpx::parallel::exclusive_scan(ex::par, in.begin(), in.end(), out.begin(), T(50));
    HPX_TEST(to_host(out) == xver);

    // task policies (inline temporaries), three algorithms in flight at once:
    // the totals and carries stay on the devices, each future completes from
    // the segments' streams
    pvec<T> out2(size, policy);
    hpx::parallel::fill(ex::par, out.begin(), out.end(), T(0));
    auto f1 = hpx::parallel::inclusive_scan(ex::par(ex::task), in.begin(), in.end(), out.begin(), std::plus<T>(), T(0));
    auto f2 =
        hpx::parallel::exclusive_scan(ex::par(ex::task), in.begin(), in.end(), out2.begin(), T(50), std::plus<T>());
    auto f3 = hpx::parallel::reduce(ex::par(ex::task), in.begin(), in.end(), T(7), std::plus<T>());
    HPX_TEST(f2.get() == out2.end());
    HPX_TEST(f1.get() == out.end());
    HPX_TEST_EQ(f3.get(), T(T(7) + ver.back()));
    HPX_TEST(to_host(out) == ver);
    HPX_TEST(to_host(out2) == xver);
    // a sub-range whose ends are inside partitions
    if (size > 20) {
        std::vector<T> sub(size - 13);
        std::partial_sum(h.begin() + 5, h.end() - 8, sub.begin());
        hpx::parallel::inclusive_scan(ex::par(ex::task), in.begin() + 5, in.end() - 8, out.begin() + 5, std::plus<T>(),
                                      T(0))
            .get();
        std::vector<T> got = to_host(out);
        HPX_TEST(std::equal(sub.begin(), sub.end(), got.begin() + 5));
    }

    // in place (inclusive_scan_tests_inplace_with_policy)
    hpx::parallel::inclusive_scan(ex::par, in.begin(), in.end(), in.begin(), std::plus<T>(), T(0));
    HPX_TEST(to_host(in) == ver);
}

void test_transform_copy(hip::target_distribution_policy const& policy) {
    std::size_t const n = 100003;
    pvec<double> a(n, 1.0, policy), b(n, 2.0, policy), c(n, policy);
    // STREAM triad over partitioned vectors
    hpx::parallel::transform(ex::par, a.begin(), a.end(), b.begin(), c.begin(), fn::triad_step<double>{3.0});
    std::vector<double> hc = to_host(c);
    HPX_TEST(std::all_of(hc.begin(), hc.end(), [](double x) { return x == 7.0; }));
    hpx::parallel::transform(ex::par(ex::task), c.begin(), c.end(), a.begin(), [] HPX_HOST_DEVICE(double x) {
        return x * 0.5;
    }).get();
    std::vector<double> ha = to_host(a);
    HPX_TEST(std::all_of(ha.begin(), ha.end(), [](double x) { return x == 3.5; }));
    hpx::parallel::copy(ex::par, a.begin(), a.end(), b.begin());
    HPX_TEST(to_host(b) == ha);
    HPX_TEST_EQ(double(a[n - 1]), 3.5);
    // sub-range reduce spanning partition boundaries
    HPX_TEST_EQ(hpx::parallel::reduce(ex::par, a.begin() + 5, a.end() - 3, 0.0), 3.5 * double(n - 8));
}

// segment order: init (+) S_0 (+) S_1 ... over the partitions (reduce.hpp:191-207)
void test_fp_segment_order(hip::target_distribution_policy const& policy) {
    std::size_t const n = 3;
    pvec<double> v(n, policy);
    std::vector<double> h = {1e16, 1.0, -1e16};
    hpx::parallel::copy(ex::par, h.begin(), h.end(), v.begin());
    double r = hpx::parallel::reduce(ex::par, v.begin(), v.end(), 1.0);
    // with one element per partition: ((1 + 1e16) + 1) + -1e16 = 0 (1e16+1 rounds to 1e16, twice)
    HPX_TEST_EQ(r, ((1.0 + 1e16) + 1.0) + -1e16);
}

int hpx_main(int, char**) {
    auto targets = hip::get_local_targets();
    std::cout << targets.size() << " HIP target(s)" << std::endl;
    std::vector<hip::target_distribution_policy> policies = {
        hip::target_layout(targets), hip::target_layout(targets, 3), hip::target_layout(targets, 1000),
        hip::target_layout(targets[0], 7)};
    for (auto const& pol : policies) {
        test_example(pol);
        test_reduce<int>(pol);
        test_reduce<double>(pol);
        test_scans<int64_t>(1000000, pol);
        test_scans<int32_t>(1000, pol);
        test_transform_copy(pol);
    }
    test_fp_segment_order(hip::target_layout(targets[0], 3));
    // every cross-stream hand-off (carries, halos) was ordered on the device
    HPX_TEST_EQ(hip::detail::stream_order_host_waits().load(), 0ul);
    return hpx::finalize();
}

int main(int argc, char* argv[]) {
    HPX_TEST_EQ(hpx::init(argc, argv), 0);
    int errors = hpx::util::report_errors();
    if (!errors) std::cout << "partitioned_vector: all tests passed" << std::endl;
    return errors;
}
