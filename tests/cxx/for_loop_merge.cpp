// C++ port of tests/unit/computeapi/cuda/for_loop_compute.cu:28-118 on the
// HIP backend (two targets, `for_loop_n(par.on(exec), A, N, induction(B),
// induction(C), *C = *A + 3.0 * *B)`, checked element by element against the
// host transform), strided inductions, for_loop reductions
// (for_loop_reduction.cpp) and for_loop_strided (for_loop_strided.cpp), task
// policies on inline temporaries, plus hpx::parallel::merge (merge.hpp:476)
// against std::merge, ascending and descending, sync and task policies.
#include <hpx/hpx.hpp>
#include <hpx/hpx_init.hpp>
#include <hpx/util/lightweight_test.hpp>

#include <algorithm>
#include <cstdint>
#include <functional>
#include <iostream>
#include <numeric>
#include <random>
#include <vector>

namespace hip = hpx::compute::hip;
namespace fn = hpx::compute::hip::functional;
namespace ex = hpx::parallel::execution;
template <typename T>
using dvec = hpx::compute::vector<T, hip::allocator<T>>;

template <typename T>
std::vector<T> to_host(dvec<T> const& d) {
    std::vector<T> h(d.size());
    hpx::parallel::copy(ex::par, d.begin(), d.end(), h.begin());
    return h;
}

void test_for_loop(std::mt19937& gen, int N) {
    std::uniform_int_distribution<> dis(2, 101);
    std::vector<int> h_A(N), h_B(N), h_C_ref(N);
    std::iota(h_A.begin(), h_A.end(), dis(gen));
    std::iota(h_B.begin(), h_B.end(), dis(gen));
    std::transform(h_A.begin(), h_A.end(), h_B.begin(), h_C_ref.begin(), [](int a, int b) { return a + 3.0 * b; });

    hip::target targetA, targetB;
    hip::allocator<int> allocA(targetA), allocB(targetB);
    dvec<int> d_A(N, allocA), d_B(N, allocB), d_C(N, allocA);
    auto f = hpx::parallel::copy(ex::par(ex::task), h_A.begin(), h_A.end(), d_A.begin());
    hpx::parallel::copy(ex::par, h_B.begin(), h_B.end(), d_B.begin());
    f.get();

    hip::default_executor exec(targetB);
    fn::loop_assign<2, fn::triad_step<double>, 0, 1> body{{3.0}};   // *C = *A + 3.0 * *B
    hpx::parallel::for_loop_n(ex::par.on(exec), d_A.begin(), d_A.size(), hpx::parallel::induction(d_B.begin()),
                              hpx::parallel::induction(d_C.begin()), body);
    std::vector<int> h_C = to_host(d_C);
    HPX_TEST_EQ(h_C.size(), h_C_ref.size());
    for (int i = 0; i < N; ++i) HPX_TEST_EQ(h_C[i], h_C_ref[i]);

    // for_loop over [first, last) under par(task), in-place unary body
    dvec<int> d_D(N, allocA);
    hpx::parallel::copy(ex::par, h_A.begin(), h_A.end(), d_D.begin());
    fn::loop_assign<0, fn::add_value<int>, 0> plus5{{5}};
    hpx::future<void> g = hpx::parallel::for_loop(ex::par(ex::task).on(exec), d_D.begin(), d_D.end(), plus5);
    g.get();
    std::vector<int> h_D = to_host(d_D);
    for (int i = 0; i < N; ++i) HPX_TEST_EQ(h_D[i], h_A[i] + 5);

    // strided induction (for_loop_induction.hpp:210-219): *C = *A + 3.0 * B[2i]
    if (N >= 2) {
        int M = N / 2;
        dvec<int> d_E(M, allocA);
        hpx::parallel::for_loop_n(ex::par.on(exec), d_A.begin(), M, hpx::parallel::induction(d_B.begin(), 2),
                                  hpx::parallel::induction(d_E.begin()), body);
        std::vector<int> h_E = to_host(d_E);
        for (int i = 0; i < M; ++i) HPX_TEST_EQ(h_E[i], static_cast<int>(h_A[i] + 3.0 * h_B[2 * i]));
    }
}

// for_loop_reduction.cpp:20-140 restated over device iterators: 10007 size_t
// iotas from a random start, `r op= *it`, checked against std::accumulate.
// Every task-form call passes its policy as an inline temporary
// (`par(task).on(exec)`): the temporary's target copy, and with it its stream,
// is gone before get() -- the result must not depend on it.
void test_for_loop_reduction(std::mt19937& gen) {
    using T = std::uint64_t;
    std::vector<T> c(10007);
    std::iota(c.begin(), c.end(), T(gen()));
    hip::target t;
    hip::allocator<T> alloc(t);
    dvec<T> d(c.size(), alloc);
    hpx::parallel::copy(ex::par, c.begin(), c.end(), d.begin());
    hip::default_executor exec(t);
    fn::loop_accumulate<1, fn::identity, 0> body{};

    T sum = 0;
    hpx::parallel::for_loop(ex::par.on(exec), d.begin(), d.end(), hpx::parallel::reduction_plus(sum), body);
    HPX_TEST_EQ(sum, std::accumulate(c.begin(), c.end(), T(0)));

    T prod = 1;
    hpx::future<void> f = hpx::parallel::for_loop(ex::par(ex::task).on(exec), d.begin(), d.end(),
                                                  hpx::parallel::reduction_multiplies(prod), body);
    f.wait();  // the live-out is final once the future is ready (for_loop_reduction.hpp:60-66)
    HPX_TEST_EQ(prod, std::accumulate(c.begin(), c.end(), T(1), std::multiplies<T>()));
    f.get();

    // many task-form reductions in flight on temporaries, read in reverse
    std::vector<T> sums(64, 0);
    std::vector<hpx::future<void>> fs;
    for (std::size_t k = 0; k < sums.size(); ++k) {
        sums[k] = k;
        fs.push_back(hpx::parallel::for_loop_n(ex::par(ex::task).on(hip::default_executor(t)), d.begin(),
                                               c.size() - k, hpx::parallel::reduction_plus(sums[k]), body));
    }
    for (std::size_t k = fs.size(); k-- > 0;) {
        fs[k].get();
        HPX_TEST_EQ(sums[k], std::accumulate(c.begin(), c.end() - k, T(k)));
    }

    std::shuffle(c.begin(), c.end(), gen);
    hpx::parallel::copy(ex::par, c.begin(), c.end(), d.begin());
    T mn = c[0], mx = c[0];
    hpx::parallel::for_loop_n(ex::par.on(exec), d.begin(), c.size(), hpx::parallel::reduction_min(mn), body);
    hpx::parallel::for_loop_n(ex::par.on(exec), d.begin(), c.size(), hpx::parallel::reduction_max(mx), body);
    HPX_TEST_EQ(mn, *std::min_element(c.begin(), c.end()));
    HPX_TEST_EQ(mx, *std::max_element(c.begin(), c.end()));

    T x = 0;
    hpx::parallel::for_loop_n(ex::par.on(exec), d.begin(), c.size(), hpx::parallel::reduction_bit_xor(x), body);
    T xr = 0;
    for (T v : c) xr ^= v;
    HPX_TEST_EQ(x, xr);

    // inner product: loop iterator and an induction feed a binary body
    std::vector<T> e(c.size(), T(3));
    dvec<T> de(e.size(), alloc);
    hpx::parallel::copy(ex::par, e.begin(), e.end(), de.begin());
    T ip = 5;
    fn::loop_accumulate<2, fn::multiply, 0, 1> dot{};
    hpx::parallel::for_loop_n(ex::par.on(exec), d.begin(), c.size(), hpx::parallel::induction(de.begin()),
                              hpx::parallel::reduction_plus(ip), dot);
    HPX_TEST_EQ(ip, std::inner_product(c.begin(), c.end(), e.begin(), T(5)));

    // several reductions in one loop (for_loop.hpp:802-812): sum, min, max
    // and the inner product with an induction, sync and task forms
    for (bool task : {false, true}) {
        T s2 = 7, lo = c[1], hi = c[1], ip2 = 11;
        auto all = fn::accumulate_all(fn::loop_accumulate<1, fn::identity, 0>{},
                                      fn::loop_accumulate<2, fn::identity, 0>{},
                                      fn::loop_accumulate<3, fn::identity, 0>{},
                                      fn::loop_accumulate<5, fn::multiply, 0, 4>{});
        auto args = [&](auto pol) {
            return hpx::parallel::for_loop_n(pol, d.begin(), c.size(), hpx::parallel::reduction_plus(s2),
                                             hpx::parallel::reduction_min(lo), hpx::parallel::reduction_max(hi),
                                             hpx::parallel::induction(de.begin()), hpx::parallel::reduction_plus(ip2),
                                             all);
        };
        if (task) {
            hpx::future<void> fa = args(ex::par(ex::task).on(exec));
            fa.get();
        } else {
            args(ex::par.on(exec));
        }
        HPX_TEST_EQ(s2, std::accumulate(c.begin(), c.end(), T(7)));
        HPX_TEST_EQ(lo, *std::min_element(c.begin(), c.end()));
        HPX_TEST_EQ(hi, *std::max_element(c.begin(), c.end()));
        HPX_TEST_EQ(ip2, std::inner_product(c.begin(), c.end(), e.begin(), T(11)));
    }
}

// Task-form reduce / transform_reduce / copy_if with inline temporary
// policies; the futures are read after the temporaries (and their streams)
// are gone, and after unrelated work reused the pooled streams.
void test_task_temporaries(std::mt19937& gen) {
    using T = std::int64_t;
    std::uniform_int_distribution<T> dis(-1000, 1000);
    std::vector<T> h(100003);
    for (auto& x : h) x = dis(gen);
    hip::target t;
    hip::allocator<T> alloc(t);
    dvec<T> d(h.size(), alloc), out(h.size(), alloc);
    hpx::parallel::copy(ex::par, h.begin(), h.end(), d.begin());

    std::vector<hpx::future<T>> rs;
    std::vector<hpx::future<hpx::parallel::util::tagged_pair<dvec<T>::iterator, dvec<T>::iterator>>> cs;
    for (int k = 0; k < 16; ++k) {
        rs.push_back(hpx::parallel::reduce(ex::par(ex::task).on(hip::default_executor(t)), d.begin(), d.end() - k,
                                           T(k)));
        rs.push_back(hpx::parallel::transform_reduce(ex::par(ex::task).on(hip::default_executor(t)), d.begin(),
                                                     d.end(), T(0), std::plus<T>(), fn::square{}));
    }
    // copy_if into one output buffer: the temporaries are created one after
    // another, each hands its stream back to the device pool as it dies and
    // the next takes it again, so the four compactions are stream-ordered
    for (int k = 0; k < 4; ++k)
        cs.push_back(hpx::parallel::copy_if(ex::par(ex::task).on(hip::default_executor(t)), d.begin(), d.end(),
                                            out.begin(), fn::greater_than<T>{T(100 * k)}));
    T sq = 0;
    for (T x : h) sq += x * x;
    for (int k = 0; k < 16; ++k) {
        HPX_TEST_EQ(rs[2 * k].get(), std::accumulate(h.begin(), h.end() - k, T(k)));
        HPX_TEST_EQ(rs[2 * k + 1].get(), sq);
    }
    for (int k = 0; k < 4; ++k) {
        auto r = cs[k].get();
        auto expect = std::count_if(h.begin(), h.end(), [k](T x) { return x > T(100 * k); });
        HPX_TEST_EQ(r.out() - out.begin(), static_cast<std::ptrdiff_t>(expect));
    }
    // the last copy_if's output is what the buffer holds
    std::vector<T> ref;
    std::copy_if(h.begin(), h.end(), std::back_inserter(ref), [](T x) { return x > T(300); });
    std::vector<T> got = to_host(out);
    got.resize(ref.size());
    HPX_TEST(got == ref);
}

// for_loop_strided.cpp:29-74 restated: every stride-th element set to 42.
void test_for_loop_strided(std::mt19937& gen) {
    using T = std::uint64_t;
    std::vector<T> c(10007);
    std::iota(c.begin(), c.end(), T(1000));
    hip::target t;
    hip::allocator<T> alloc(t);
    hip::default_executor exec(t);
    for (int stride : {1, 2, 7, int(gen() % 100) + 1, 10007, 20000}) {
        dvec<T> d(c.size(), alloc);
        hpx::parallel::copy(ex::par, c.begin(), c.end(), d.begin());
        fn::loop_assign<0, fn::affine<T>, 0> set42{{T(0), T(42)}};
        hpx::parallel::for_loop_strided(ex::par.on(exec), d.begin(), d.end(), stride, set42);
        std::vector<T> h = to_host(d);
        for (std::size_t i = 0; i != h.size(); ++i) {
            if (i % stride == 0) HPX_TEST_EQ(h[i], T(42));
            else HPX_TEST_NEQ(h[i], T(42));
        }
        // same through a task policy on a temporary
        hpx::parallel::copy(ex::par, c.begin(), c.end(), d.begin());
        hpx::parallel::for_loop_strided(ex::par(ex::task).on(hip::default_executor(t)), d.begin(), d.end(), stride,
                                        set42)
            .get();
        h = to_host(d);
        for (std::size_t i = 0; i != h.size(); ++i)
            if (i % stride == 0) HPX_TEST_EQ(h[i], T(42));
    }
}

template <typename T, typename Comp>
void test_merge(std::mt19937& gen, std::size_t n1, std::size_t n2, Comp comp) {
    std::uniform_int_distribution<int> dis(0, 50);
    std::vector<T> a(n1), b(n2);
    for (auto& x : a) x = static_cast<T>(dis(gen));
    for (auto& x : b) x = static_cast<T>(dis(gen));
    std::sort(a.begin(), a.end(), comp);
    std::sort(b.begin(), b.end(), comp);
    std::vector<T> ref(n1 + n2);
    std::merge(a.begin(), a.end(), b.begin(), b.end(), ref.begin(), comp);
    hip::target t;
    hip::allocator<T> alloc(t);
    dvec<T> da(n1, alloc), db(n2, alloc), dout(n1 + n2, alloc);
    hpx::parallel::copy(ex::par, a.begin(), a.end(), da.begin());
    hpx::parallel::copy(ex::par, b.begin(), b.end(), db.begin());
    hip::default_executor exec(t);
    auto r = hpx::parallel::merge(ex::par.on(exec), da.begin(), da.end(), db.begin(), db.end(), dout.begin(), comp);
    HPX_TEST(r.out() == dout.end());
    std::vector<T> got = to_host(dout);
    HPX_TEST(got == ref);
    auto fr = hpx::parallel::merge(ex::par(ex::task).on(exec), da.begin(), da.end(), db.begin(), db.end(),
                                   dout.begin(), comp);
    HPX_TEST(fr.get().in1() == da.end());
}

int hpx_main(int, char**) {
    std::mt19937 gen(42);
    for (int n : {100, 1, 4097, 1 << 20}) test_for_loop(gen, n);
    test_for_loop_reduction(gen);
    test_task_temporaries(gen);
    test_for_loop_strided(gen);
    test_merge<int64_t>(gen, 10007, 5003, std::less<int64_t>());
    test_merge<uint32_t>(gen, 1 << 20, (1 << 19) + 3, std::greater<uint32_t>());
    test_merge<double>(gen, 4096, 0, std::less<double>());
    return hpx::finalize();
}

int main(int argc, char* argv[]) {
    HPX_TEST_EQ(hpx::init(argc, argv), 0);
    int errors = hpx::util::report_errors();
    if (!errors) std::cout << "for_loop_merge: all tests passed" << std::endl;
    return errors;
}
