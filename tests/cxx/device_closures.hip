// Device closures through the HIP backend's HPX C++ layer, compiled by hipcc:
// the reference's GPU tests with their ORIGINAL callables (no trait
// specialisation), the executor concept, and the concurrent executor.
//
//   for_each_compute.cu:28-51    for_each(par.on(exec), ..., [] HPX_HOST_DEVICE (int& i) { i += 5; })
//   transform_compute.cu:28-63   transform(par.on(exec), A, A_end, B, C, transform_test())
//   for_loop_compute.cu:28-118   for_loop_n(par.on(exec), A.data(), N, induction(B.data()),
//                                           induction(C.data()), [] HPX_HOST_DEVICE (int* A, int* B, int* C)
//                                           { *C = *A + 3.0 * *B; })
//   default_executor.cu:20-97    sync_execute / async_execute / bulk_sync_execute /
//                                bulk_async_execute over a 107-element shape
//   concurrent_executor.hpp      the same over several streams, plus the
//                                elementwise algorithms chunked over its streams
//
// usage: device_closures [seed]
#include <hpx/hpx.hpp>
#include <hpx/hpx_init.hpp>
#include <hpx/util/lightweight_test.hpp>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <iostream>
#include <numeric>
#include <random>
#include <vector>

namespace hip = hpx::compute::hip;
namespace ex = hpx::parallel::execution;
using executor_type = hip::default_executor;
using target_allocator = hip::allocator<int>;
using target_vector = hpx::compute::vector<int, target_allocator>;

template <typename T, typename A>
std::vector<T> to_host(hpx::compute::vector<T, A> const& d) {
    std::vector<T> h(d.size());
    hpx::parallel::copy(ex::par, d.begin(), d.end(), h.begin());
    return h;
}

// ---------------------------------------------------------- for_each_compute.cu
void test_for_each(executor_type& exec, target_vector& d_A) {
    std::vector<int> h_C(d_A.size());
    hpx::parallel::copy(ex::par, d_A.begin(), d_A.end(), h_C.begin());
    hpx::parallel::for_each(ex::par.on(exec), d_A.begin(), d_A.end(), [] HPX_HOST_DEVICE(int& i) { i += 5; });
    for (std::size_t i = 0; i != h_C.size(); ++i) {
        if (!HPX_TEST_EQ(h_C[i] + 5, d_A[i])) break;
    }
}

// --------------------------------------------------------- transform_compute.cu
struct transform_test {
    template <typename T>
    HPX_HOST_DEVICE int operator()(T const& a, T const& b) const {
        return a + 3.0 * b;
    }
};
void test_transform(executor_type& exec, target_vector& d_A, target_vector& d_B, target_vector& d_C,
                    std::vector<int> const& ref) {
    hpx::parallel::transform(ex::par.on(exec), d_A.begin(), d_A.end(), d_B.begin(), d_C.begin(), transform_test());
    std::vector<int> h_C = to_host(d_C);
    HPX_TEST_EQ(h_C.size(), ref.size());
    for (std::size_t i = 0; i != ref.size(); ++i)
        if (!HPX_TEST_EQ(h_C[i], ref[i])) break;
}

// ---------------------------------------------------------- for_loop_compute.cu
void test_for_loop(executor_type& exec, target_vector& d_A, target_vector& d_B, target_vector& d_C,
                   std::vector<int> const& ref) {
    hpx::parallel::for_loop_n(ex::par.on(exec), d_A.data(), d_A.size(), hpx::parallel::induction(d_B.data()),
                              hpx::parallel::induction(d_C.data()),
                              [] HPX_HOST_DEVICE(int* A, int* B, int* C) { *C = *A + 3.0 * *B; });
    std::vector<int> h_C = to_host(d_C);
    HPX_TEST_EQ(h_C.size(), ref.size());
    for (std::size_t i = 0; i != ref.size(); ++i) {
        if (!HPX_TEST_EQ(h_C[i], ref[i])) break;
        if (i < 8) HPX_TEST_EQ(d_C[i], ref[i]);  // value_proxy reads
    }
}

void run_compute_tests(std::mt19937& gen) {
    std::uniform_int_distribution<> dis(2, 101);
    for (int N : {100, 10007, (1 << 20) + 3}) {
        std::vector<int> h_A(N), h_B(N), ref(N);
        std::iota(h_A.begin(), h_A.end(), dis(gen));
        std::iota(h_B.begin(), h_B.end(), dis(gen));
        std::transform(h_A.begin(), h_A.end(), h_B.begin(), ref.begin(), [](int a, int b) { return a + 3.0 * b; });

        hip::target targetA, targetB;
        target_allocator allocA(targetA), allocB(targetB);
        target_vector d_A(N, allocA), d_B(N, allocB), d_C(N, allocA);
        auto f = hpx::parallel::copy(ex::par(ex::task), h_A.begin(), h_A.end(), d_A.begin());
        hpx::parallel::copy(ex::par, h_B.begin(), h_B.end(), d_B.begin());
        f.get();
        executor_type exec(targetB);
        test_for_loop(exec, d_A, d_B, d_C, ref);
        hpx::parallel::fill(ex::par, d_C.begin(), d_C.end(), 0);
        test_transform(exec, d_A, d_B, d_C, ref);
        test_for_each(exec, d_A);
    }
}

// ---------------------------------------------------------- default_executor.cu
// The reference's closures are empty (`__device__ void operator()() {}`);
// these write what they did so the test can check it ran on the device.
struct test {
    int* flag;
    __device__ void operator()() { atomicAdd(flag, 1); }
};
struct bulk_test {
    int* out;
    int base;
    HPX_HOST_DEVICE void operator()(int i) { out[i - base] = 2 * i + 1; }
};
// slow on purpose: ~1000 dependent steps per element
struct bulk_slow {
    int* out;
    int iters = 1000;
    HPX_HOST_DEVICE static int expect(int i, int iters = 1000) {
        uint32_t x = uint32_t(i);
        for (int k = 0; k < iters; ++k) x = x * 1664525u + 1013904223u;
        return int(x >> 1);
    }
    HPX_HOST_DEVICE void operator()(int i) { out[i - 3] = expect(i, iters); }
};
// Waits (bounded: ~3 s, then runs anyway) until the host opens the gate, a
// word in pinned host memory: the work is certainly pending until then.
struct bulk_gated {
    int* out;
    int const* gate;
    __device__ static bool open(int const* g) {
        return __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0;
    }
    HPX_HOST_DEVICE void operator()(int i) {
#if defined(__HIP_DEVICE_COMPILE__)
        for (int spins = 0; spins < (1 << 20) && !open(gate); ++spins) __builtin_amdgcn_s_sleep(127);
#endif
        out[i - 3] = bulk_slow::expect(i, 16);
    }
};
struct bulk_test_args {
    HPX_HOST_DEVICE void operator()(int i, int* out, int base, int add) { out[i - base] = i + add; }
};

template <typename Executor>
void test_executor(Executor& exec, hip::target const& t, std::mt19937& gen, char const* name) {
    static_assert(ex::is_one_way_executor<Executor>::value && ex::is_two_way_executor<Executor>::value &&
                      ex::is_bulk_one_way_executor<Executor>::value && ex::is_bulk_two_way_executor<Executor>::value,
                  "executor traits");
    static_assert(std::is_same<typename ex::executor_execution_category<Executor>::type,
                               ex::parallel_execution_tag>::value,
                  "parallel execution category");
    HPX_TEST(exec.processing_units_count() > 0);
    std::cout << name << ": " << exec.processing_units_count() << " processing units" << std::endl;

    hip::allocator<int> alloc(t);
    hpx::compute::vector<int, hip::allocator<int>> flag(1, 0, alloc);
    ex::sync_execute(exec, test{flag.data()});  // test_sync
    HPX_TEST_EQ(int(flag[0]), 1);
    ex::async_execute(exec, test{flag.data()}).get();  // test_async
    HPX_TEST_EQ(int(flag[0]), 2);
    exec.post(test{flag.data()});
    exec.sync_execute(test{flag.data()});
    if constexpr (std::is_same<Executor, hip::concurrent_executor>::value) exec.synchronize();
    HPX_TEST_EQ(int(flag[0]), 4);

    std::vector<int> v(107);  // test_bulk_sync / test_bulk_async
    int base = static_cast<int>(gen() % 100000);
    std::iota(v.begin(), v.end(), base);
    hpx::compute::vector<int, hip::allocator<int>> out(v.size(), -1, alloc);
    ex::bulk_sync_execute(exec, bulk_test{out.data(), base}, v);
    std::vector<int> h = to_host(out);
    for (std::size_t i = 0; i != v.size(); ++i) HPX_TEST_EQ(h[i], 2 * v[i] + 1);

    hpx::parallel::fill(ex::par, out.begin(), out.end(), -1);
    hpx::when_all(ex::bulk_async_execute(exec, bulk_test_args{}, v, out.data(), base, 7)).get();
    h = to_host(out);
    for (std::size_t i = 0; i != v.size(); ++i) HPX_TEST_EQ(h[i], v[i] + 7);

    // 10^6-element bulk_async_execute: the shape is staged (pinned, pooled)
    // and the call returns while the device still works; every element ran
    // exactly once, the shape's first element included
    std::vector<int> big(1000000);
    std::iota(big.begin(), big.end(), 3);
    hpx::compute::vector<int, hip::allocator<int>> bo(big.size(), -1, alloc);
    {
        // the body waits for a gate the host opens only after checking that
        // the futures are pending (r05: deterministic; r04 raced a slow
        // kernel's duration against the host building 10^6 futures)
        int* gate = nullptr;
        HPX_TEST_EQ(hpxhip_malloc_host(reinterpret_cast<void**>(&gate), sizeof(int)), 0);
        __atomic_store_n(gate, 0, __ATOMIC_SEQ_CST);
        auto fs = ex::bulk_async_execute(exec, bulk_gated{bo.data(), gate}, big);
        bool pending = true;
        for (auto& f : fs) pending = pending && !f.is_ready();
        HPX_TEST(pending);
        big.assign(big.size(), 0);  // the caller's shape may go away at once
        __atomic_store_n(gate, 1, __ATOMIC_SEQ_CST);
        hpx::when_all(std::move(fs)).get();
        std::vector<int> hb = to_host(bo);
        for (std::size_t i = 0; i != hb.size(); ++i)
            if (!HPX_TEST_EQ(hb[i], bulk_slow::expect(int(i) + 3, 16))) break;
        hpxhip_free_host(gate);
    }
    std::iota(big.begin(), big.end(), 3);
    auto fs = ex::bulk_async_execute(exec, bulk_slow{bo.data()}, big);
    // cuda default_executor: one future for the bulk launch (:196-210);
    // concurrent_executor: one future per shape element (:171-193)
    if constexpr (std::is_same<Executor, hip::concurrent_executor>::value) HPX_TEST_EQ(fs.size(), big.size());
    else HPX_TEST_EQ(fs.size(), std::size_t(1));
    big.assign(big.size(), 0);
    hpx::when_all(std::move(fs)).get();
    std::vector<int> hb = to_host(bo);
    for (std::size_t i = 0; i != hb.size(); ++i)
        if (!HPX_TEST_EQ(hb[i], bulk_slow::expect(int(i) + 3))) break;
}

// ------------------------------------------------ concurrent_executor algorithms
void test_concurrent_algorithms(std::mt19937& gen) {
    hip::target t;
    hip::concurrent_executor cexec(t, 4);
    HPX_TEST_EQ(cexec.processing_units_count(), std::size_t(4));
    using T = double;
    hip::allocator<T> alloc(t);
    for (std::size_t n : {std::size_t(1), std::size_t(3), std::size_t(1000003)}) {
        hpx::compute::vector<T, hip::allocator<T>> a(n, alloc), b(n, alloc), c(n, alloc);
        auto pol = ex::par.on(cexec);
        hpx::parallel::fill(pol, a.begin(), a.end(), 1.0);
        hpx::parallel::fill(pol, b.begin(), b.end(), 2.0);
        // STREAM triad on the concurrent executor (stream.cpp:428-453)
        hpx::parallel::transform(pol, b.begin(), b.end(), a.begin(), c.begin(), hip::functional::triad_step<T>{3.0});
        std::vector<T> hc = to_host(c);
        HPX_TEST(std::all_of(hc.begin(), hc.end(), [](T x) { return x == 5.0; }));
        // a device lambda chunked over the streams, task policy
        hpx::parallel::for_each(ex::par(ex::task).on(cexec), c.begin(), c.end(), [] HPX_HOST_DEVICE(T & x) {
            x = x * 2.0 + 1.0;
        }).get();
        hc = to_host(c);
        HPX_TEST(std::all_of(hc.begin(), hc.end(), [](T x) { return x == 11.0; }));
        // single-kernel algorithms run on the first stream
        T s = hpx::parallel::reduce(pol, c.begin(), c.end(), T(0));
        HPX_TEST_EQ(s, 11.0 * T(n));
    }
    // integer for_loop with a raw-pointer lambda on the concurrent executor
    std::vector<int64_t> h(12345);
    std::iota(h.begin(), h.end(), int64_t(gen() % 1000));
    hip::allocator<int64_t> ai(t);
    hpx::compute::vector<int64_t, hip::allocator<int64_t>> d(h.size(), ai), e(h.size(), ai);
    hpx::parallel::copy(ex::par, h.begin(), h.end(), d.begin());
    hpx::parallel::for_loop_n(ex::par.on(cexec), d.data(), h.size(), hpx::parallel::induction(e.data()),
                              [] HPX_HOST_DEVICE(int64_t * x, int64_t * y) { *y = *x * *x - 3; });
    std::vector<int64_t> he = to_host(e);
    for (std::size_t i = 0; i != h.size(); ++i)
        if (!HPX_TEST_EQ(he[i], h[i] * h[i] - 3)) break;
}

// for_loop with a lambda body and reductions (for_loop_reduction.hpp:35-132,
// for_loop_reduction.cpp's bodies with device iterators): each reduction
// reaches the body as a reference to a private view; several reductions and
// an induction in one loop, sync and task forms, an empty loop.
void test_for_loop_lambda_reductions(std::mt19937& gen) {
    using T = int64_t;
    std::vector<T> h(1000003), g(h.size());
    std::uniform_int_distribution<T> dis(-1000, 1000);
    for (auto& x : h) x = dis(gen);
    for (auto& x : g) x = dis(gen);
    hip::target t;
    hip::allocator<T> a(t);
    hpx::compute::vector<T, hip::allocator<T>> d(h.size(), a), e(g.size(), a);
    hpx::parallel::copy(ex::par, h.begin(), h.end(), d.begin());
    hpx::parallel::copy(ex::par, g.begin(), g.end(), e.begin());
    hip::default_executor exec(t);
    for (bool task : {false, true}) {
        T sum = 3, mx = h[0], dot = -5;
        uint64_t odd = 0;
        auto body = [] HPX_HOST_DEVICE(T * x, T & s, T & m, T * y, T & dp, uint64_t & o) {
            s += *x;
            m = *x > m ? *x : m;
            dp += *x * *y;
            o += (*x & 1) ? 1u : 0u;
        };
        auto run = [&](auto pol) {
            return hpx::parallel::for_loop_n(pol, d.data(), h.size(), hpx::parallel::reduction_plus(sum),
                                             hpx::parallel::reduction_max(mx), hpx::parallel::induction(e.data()),
                                             hpx::parallel::reduction_plus(dot), hpx::parallel::reduction_plus(odd),
                                             body);
        };
        if (task) {
            hpx::future<void> f = run(ex::par(ex::task).on(exec));
            f.wait();  // the live-outs are final once the future is ready
            f.get();
        } else {
            run(ex::par.on(exec));
        }
        HPX_TEST_EQ(sum, std::accumulate(h.begin(), h.end(), T(3)));
        HPX_TEST_EQ(mx, *std::max_element(h.begin(), h.end()));
        HPX_TEST_EQ(dot, std::inner_product(h.begin(), h.end(), g.begin(), T(-5)));
        HPX_TEST_EQ(odd, uint64_t(std::count_if(h.begin(), h.end(), [](T x) { return (x & 1) != 0; })));
    }
    // an empty loop leaves every live-out at var (op) identity
    double p = 2.5;
    hpx::parallel::for_loop_n(ex::par.on(exec), d.data(), 0, hpx::parallel::reduction_multiplies(p),
                              [] HPX_HOST_DEVICE(T * x, double& q) { q *= double(*x); });
    HPX_TEST_EQ(p, 2.5);
}

int hpx_main(int argc, char* argv[]) {
    unsigned seed = argc > 1 ? unsigned(std::strtoul(argv[1], nullptr, 10)) : std::random_device{}();
    std::cout << "using seed: " << seed << std::endl;
    std::mt19937 gen(seed);
    run_compute_tests(gen);

    hip::target target;
    executor_type exec(target);
    test_executor(exec, target, gen, "default_executor");
    hip::concurrent_executor cexec(target, 3);
    test_executor(cexec, target, gen, "concurrent_executor");
    test_concurrent_algorithms(gen);
    test_for_loop_lambda_reductions(gen);
    return hpx::finalize();
}

int main(int argc, char* argv[]) {
    HPX_TEST_EQ(hpx::init(argc, argv), 0);
    int errors = hpx::util::report_errors();
    if (!errors) std::cout << "device_closures: all tests passed" << std::endl;
    return errors;
}
