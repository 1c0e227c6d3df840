// C++ drop-in check of the HIP backend's HPX compute API: the shape of the
// reference's tests/unit/computeapi/cuda/{for_each_compute,transform_compute}.cu
// (target, allocator, compute::vector, default_executor, par.on(exec),
// copy to and from the host, value_proxy element access), plus futures from
// task policies (cuda_future.cpp) and the error paths.
//
// Built against include/ and hpx_amd/libhpxhip.so by `make cxxtests`; run by
// tests/test_cxx_api.py under pytest -m gpu.
#include <memory>
#include <hpx/hpx.hpp>
#include <hpx/hpx_init.hpp>
#include <hpx/util/lightweight_test.hpp>

#include <cstdint>
#include <cstdlib>
#include <iostream>
#include <numeric>
#include <random>
#include <vector>

using executor_type = hpx::compute::hip::default_executor;
using target_allocator = hpx::compute::hip::allocator<int>;
using target_vector = hpx::compute::vector<int, target_allocator>;
namespace fn = hpx::compute::hip::functional;
namespace ex = hpx::parallel::execution;

// transform_compute.cu:29-40 defines `int operator()(a, b) { return a + 3.0 * b; }`;
// a user functor reaches the device by declaring which built-in op it is.
struct transform_test {
    template <typename T>
    int operator()(T const& a, T const& b) const {
        return a + 3.0 * b;
    }
};
template <>
struct hpx::compute::hip::traits::binary<transform_test> {
    static constexpr int kind = HPXHIP_B_TRIAD;
    using compute_type = double;
    template <typename C>
    static void scalars(transform_test const&, C* s) {
        s[0] = C(3.0);
    }
};

// for_each_compute.cu:40 `i += 5`
void test_for_each(executor_type& exec, target_vector& d_A) {
    std::vector<int> h_C(d_A.size());
    hpx::parallel::copy(ex::par, d_A.begin(), d_A.end(), h_C.begin());
    hpx::parallel::for_each(ex::par.on(exec), d_A.begin(), d_A.end(), fn::add_value<int>{5});
    std::vector<int> h_A(d_A.size());
    hpx::parallel::copy(ex::par, d_A.begin(), d_A.end(), h_A.begin());
    for (std::size_t i = 0; i != h_C.size(); ++i) {
        if (!HPX_TEST_EQ(h_C[i] + 5, h_A[i])) break;
        if (i < 16) HPX_TEST_EQ(h_C[i] + 5, d_A[i]);  // value_proxy reads (one D2H each)
    }
}

void test_transform(executor_type& exec, target_vector& d_A, target_vector& d_B, target_vector& d_C,
                    std::vector<int> const& ref) {
    auto r = hpx::parallel::transform(ex::par.on(exec), d_A.begin(), d_A.end(), d_B.begin(), d_C.begin(),
                                      transform_test());
    HPX_TEST(r.out() == d_C.end());
    HPX_TEST(r.in1() == d_A.end());
    std::vector<int> h_C(d_C.size());
    hpx::parallel::copy(ex::par, d_C.begin(), d_C.end(), h_C.begin());
    HPX_TEST_EQ(h_C.size(), ref.size());
    HPX_TEST_EQ(d_C.size(), ref.size());
    for (std::size_t i = 0; i != ref.size(); ++i) {
        if (!HPX_TEST_EQ(h_C[i], ref[i])) break;
        if (i < 16) HPX_TEST_EQ(d_C[i], ref[i]);  // value_proxy reads (one D2H each)
    }
}

void test_targets_and_vector() {
    auto targets = hpx::compute::hip::get_local_targets();
    HPX_TEST(!targets.empty());
    hpx::compute::hip::target t;
    HPX_TEST(t.processing_units() > 0);
    HPX_TEST(t.native_handle().get_stream() != nullptr);

    hpx::compute::hip::allocator<double> alloc(t);
    HPX_TEST(alloc.max_size() > (std::size_t(1) << 30));
    hpx::compute::vector<double, hpx::compute::hip::allocator<double>> v(1000, 2.5, alloc);
    HPX_TEST_EQ(v.size(), std::size_t(1000));
    HPX_TEST_EQ(double(v[999]), 2.5);
    v[3] = 7.0;
    HPX_TEST_EQ(double(v[3]), 7.0);
    hpx::compute::vector<double, hpx::compute::hip::allocator<double>> z(17, alloc);  // value-initialised
    HPX_TEST_EQ(double(z[16]), 0.0);
    // move keeps the allocation
    auto moved = std::move(v);
    HPX_TEST_EQ(moved.size(), std::size_t(1000));
    HPX_TEST_EQ(double(moved[3]), 7.0);

    // ownership edge cases: a moved-from target keeps a usable handle (it
    // shares the stream), iterators taken before a vector is moved stay valid
    // after the moved-from vector is gone, and move assignment frees the old
    // allocation and takes the new one with its target
    hpx::compute::hip::target t1;
    hpx::compute::hip::target t2(std::move(t1));
    HPX_TEST_EQ(t1.device(), t2.device());
    HPX_TEST(t1.stream() != nullptr);
    HPX_TEST(t1.stream() == t2.stream());
    t1.synchronize();
    hpx::compute::hip::target t3;
    t3 = std::move(t2);
    HPX_TEST(t3.stream() == t1.stream());
    using dvec = hpx::compute::vector<double, hpx::compute::hip::allocator<double>>;
    auto pv = std::make_unique<dvec>(4096, 0.5, alloc);
    auto b = pv->begin(), e = pv->end();
    dvec w(std::move(*pv));
    pv.reset();  // the moved-from vector (and its allocator object) is gone
    HPX_TEST(b == w.begin() && e == w.end());
    HPX_TEST(b.target().stream() == w.begin().target().stream());
    HPX_TEST_EQ(hpx::parallel::reduce(ex::par, b, e, 0.0), 2048.0);
    HPX_TEST_EQ(double(b[4095]), 0.5);
    dvec u(8, 1.0, alloc);
    u = std::move(w);
    HPX_TEST_EQ(u.size(), std::size_t(4096));
    HPX_TEST(w.size() == 0 && w.data() == nullptr);
    HPX_TEST_EQ(hpx::parallel::reduce(ex::par, u.begin(), u.end(), 0.0), 2048.0);
}

void test_futures(executor_type& exec) {
    hpx::compute::hip::target t;
    hpx::compute::hip::allocator<double> alloc(t);
    std::size_t const n = 1 << 20;
    hpx::compute::vector<double, hpx::compute::hip::allocator<double>> a(n, 1.0, alloc), b(n, 2.0, alloc),
        c(n, alloc);
    hpx::compute::hip::default_executor dexec(t);
    auto pol = ex::par(ex::task).on(dexec);

    hpx::future<void> f = hpx::parallel::fill(pol, c.begin(), c.end(), 0.5);
    f.get();
    auto tf = hpx::parallel::transform(pol, a.begin(), a.end(), b.begin(), c.begin(), fn::triad_step<double>{3.0});
    auto r = tf.get();
    HPX_TEST(r.out() == c.end());
    HPX_TEST_EQ(double(c[n - 1]), 7.0);

    // reduce as a future, chained with then()
    hpx::future<double> s = hpx::parallel::reduce(pol, c.begin(), c.end(), 0.0);
    auto twice = s.then([](hpx::future<double>& x) { return 2.0 * x.get(); });
    HPX_TEST_EQ(twice.get(), 14.0 * double(n));

    // target future: ready once all work queued on that target's stream is
    // done.  The policy holds its own copy of the executor (and so of the
    // target, with its own stream, cuda_target.cpp:203-211): the kernel runs
    // on pol's stream, so that is the target whose future orders the read.
    auto fe = hpx::parallel::for_each(pol, c.begin(), c.end(), fn::multiply_step<double>{0.5});
    auto tgt_done = pol.executor().target().get_future();
    tgt_done.get();
    HPX_TEST(tgt_done.is_ready());
    fe.get();
    HPX_TEST_EQ(double(c[0]), 3.5);

    // when_all over futures of independent reductions
    std::vector<hpx::future<double>> fs;
    fs.push_back(hpx::parallel::reduce(pol, a.begin(), a.end(), 0.0));
    fs.push_back(hpx::parallel::reduce(pol, b.begin(), b.end(), 0.0));
    auto all = hpx::when_all(std::move(fs)).get();
    HPX_TEST_EQ(all[0].get(), double(n));
    HPX_TEST_EQ(all[1].get(), 2.0 * double(n));

    auto ready = hpx::make_ready_future(42);
    HPX_TEST_EQ(ready.get(), 42);
    (void)exec;
}

// Completion paths of device futures:
//   - futures dropped before their work finished hand slot and event to the
//     pool, then more reductions than one 256-slot chunk holds;
//   - when_all(...).then(...).get() over device futures (armed group);
//   - is_ready() polled on a future armed by a continuation;
//   - dataflow(unwrapping(f), device futures...) and a shared_future read by
//     two continuations;
//   - an event wait that fails (injected): get() reports exception_list with
//     the HIP status, and a second get() reports it again instead of hanging.
void test_completion_paths() {
    hpx::compute::hip::target t;
    hpx::compute::hip::allocator<double> alloc(t);
    std::size_t const n = 1 << 22;
    hpx::compute::vector<double, hpx::compute::hip::allocator<double>> a(n, 1.0, alloc), b(n, 2.0, alloc);
    hpx::compute::hip::default_executor dexec(t);
    auto pol = ex::par(ex::task).on(dexec);

    for (int i = 0; i < 64; ++i) (void)hpx::parallel::reduce(pol, a.begin(), a.end(), 0.0);  // dropped at once
    std::vector<hpx::future<double>> many;
    for (int i = 0; i < 600; ++i) many.push_back(hpx::parallel::reduce(pol, (i & 1) ? a.begin() : b.begin(),
                                                                       (i & 1) ? a.end() : b.end(), double(i)));
    bool all_ok = true;
    for (int i = 0; i < 600; ++i) all_ok &= many[i].get() == double(i) + ((i & 1) ? 1.0 : 2.0) * double(n);
    HPX_TEST(all_ok);

    std::vector<hpx::future<double>> fs;
    for (int i = 0; i < 6; ++i) fs.push_back(hpx::parallel::reduce(pol, a.begin(), a.end(), double(i)));
    auto sum = hpx::when_all(std::move(fs)).then([](hpx::future<std::vector<hpx::future<double>>> all) {
        double s = 0;
        for (auto& f : all.get()) s += f.get();
        return s;
    });
    HPX_TEST_EQ(sum.get(), 6.0 * double(n) + 15.0);

    hpx::future<double> armed = hpx::parallel::reduce(pol, b.begin(), b.end(), 0.0);
    hpx::shared_future<double> shared = armed.share();
    auto c1 = shared.then([](hpx::shared_future<double> f) { return f.get() + 1.0; });
    auto c2 = shared.then([](hpx::shared_future<double> const& f) { return f.get() + 2.0; });
    long polls = 0;
    while (!c1.is_ready()) ++polls;  // armed: the completion engine readies it
    HPX_TEST_EQ(c1.get(), 2.0 * double(n) + 1.0);
    HPX_TEST_EQ(c2.get(), 2.0 * double(n) + 2.0);
    HPX_TEST(shared.is_ready());
    std::cout << "  is_ready() polls until the armed continuation ran: " << polls << std::endl;

    auto df = hpx::dataflow(hpx::util::unwrapping([](double x, double y) { return x * y; }),
                            hpx::parallel::reduce(pol, a.begin(), a.end(), 0.0),
                            hpx::parallel::reduce(pol, b.begin(), b.end(), 0.0));
    HPX_TEST_EQ(df.get(), double(n) * 2.0 * double(n));

    hpx::future<double> failing = hpx::parallel::reduce(pol, a.begin(), a.end(), 0.0);
    HPX_TEST_EQ(hpxhip_debug_inject_event_error(709 /* hipErrorContextIsDestroyed */, 1), 0);
    int caught = 0;
    for (int k = 0; k < 2; ++k) {
        try {
            (void)failing.get();
        } catch (hpx::exception_list const& e) {
            caught += e.status == 709 ? 1 : 0;
        }
    }
    HPX_TEST_EQ(hpxhip_debug_inject_event_error(0, 0), 0);
    HPX_TEST_EQ(caught, 2);
    // the stream and the pools still work afterwards
    HPX_TEST_EQ(hpx::parallel::reduce(pol, a.begin(), a.end(), 1.0).get(), double(n) + 1.0);
}

void test_errors() {
    hpx::compute::hip::target t;
    hpx::compute::hip::allocator<float> alloc(t);
    bool threw = false;
    try {
        (void)alloc.allocate(std::size_t(1) << 60);  // far beyond HBM
    } catch (hpx::out_of_memory const&) {
        threw = true;
    } catch (std::bad_alloc const&) {
        threw = true;
    }
    HPX_TEST(threw);

    // reduce conversion not built for reductions (NEGATE) -> an error, not a
    // host fallback; algorithms report it as hpx::exception_list holding the
    // kernel_error (dispatch.hpp:122-124; tests/cxx/exception_list.cpp)
    hpx::compute::vector<float, hpx::compute::hip::allocator<float>> v(64, 1.0f, alloc);
    threw = false;
    try {
        (void)hpx::parallel::transform_reduce(ex::par, v.begin(), v.end(), 0.0f, std::plus<float>(), fn::negate{});
    } catch (hpx::exception_list const& e) {
        threw = (e.status == HPXHIP_ERROR_UNSUPPORTED && e.size() == 1);
    }
    HPX_TEST(threw);
}

// value_proxy from a temporary iterator: the proxy holds a view
// of the container's target handle, not a pointer into the iterator, so it
// stays usable after the iterator is gone; iterators are trivially copyable
// (device closures may capture them).
void test_proxy_outlives_iterator() {
    static_assert(std::is_trivially_copyable<target_vector::iterator>::value, "iterator: two pointers");
    target_vector v(16, 7);
    auto r = *v.begin();
    int x = r;
    HPX_TEST_EQ(x, 7);
    auto w = (v.begin() + 3)[0];
    w = 42;
    HPX_TEST_EQ(int(v[3]), 42);
    HPX_TEST_EQ(int(*(v.begin() + 3)), 42);
    target_vector moved(std::move(v));
    auto it = moved.begin() + 3;
    HPX_TEST_EQ(int(*it), 42);
}

int hpx_main(int argc, char* argv[]) {
    unsigned seed = argc > 1 ? unsigned(std::strtoul(argv[1], nullptr, 10)) : std::random_device{}();
    std::cout << "using seed: " << seed << std::endl;
    std::mt19937 gen(seed);
    std::uniform_int_distribution<> dis(2, 101);

    test_proxy_outlives_iterator();
    test_completion_paths();
    for (int N : {100, 10007, 1 << 20}) {
        std::vector<int> h_A(N), h_B(N);
        std::iota(h_A.begin(), h_A.end(), dis(gen));
        std::iota(h_B.begin(), h_B.end(), dis(gen));

        hpx::compute::hip::target target;
        target_allocator alloc(target);
        target_vector d_A(N, alloc), d_B(N, alloc), d_C(N, alloc);
        hpx::parallel::copy(ex::par, h_A.begin(), h_A.end(), d_A.begin());
        hpx::parallel::copy(ex::par, h_B.begin(), h_B.end(), d_B.begin());

        std::vector<int> ref(N);
        std::transform(h_A.begin(), h_A.end(), h_B.begin(), ref.begin(), transform_test());

        executor_type exec(target);
        test_transform(exec, d_A, d_B, d_C, ref);
        test_for_each(exec, d_A);
    }
    test_targets_and_vector();
    executor_type exec;
    test_futures(exec);
    test_errors();
    return hpx::finalize();
}

int main(int argc, char* argv[]) {
    HPX_TEST_EQ(hpx::init(argc, argv), 0);
    int errors = hpx::util::report_errors();
    if (!errors) std::cout << "compute_api: all tests passed" << std::endl;
    return errors;
}
