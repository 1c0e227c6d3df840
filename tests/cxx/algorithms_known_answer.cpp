// Known-answer tests of the reference's algorithm suite, restated against the
// HIP backend's C++ layer:
//
//   exclusive_scan_validate.cpp:46-131  closed forms (triangle numbers, n*x),
//                                       out of place and in place
//   inclusive_scan_tests.hpp:26-60      N x 1.0 doubles, exact; 10007 x size_t(1)
//   copyif_random.cpp:27-63             half >= 0, half < 0, `!(i < 0)`
//   partitioned_vector_reduce.cpp:47-76 10007 ones + init 1 = 10008 (int, double)
//   transform_reduce_binary (inner product) of iota vectors
//   sort_tests.hpp:122-145              sortedness (ascending, descending),
//                                       sort_by_key stability
//   fill / fill_n / copy_n / for_each_n result iterators
//
// Every check compares against a host computation with the C++ standard
// library on the same inputs; integers are bit-exact.
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
namespace fn = hpx::compute::hip::functional;
namespace ex = hpx::parallel::execution;
template <typename T>
using dvec = hpx::compute::vector<T, hip::allocator<T>>;

static std::mt19937_64 gen;

template <typename T>
std::vector<T> to_host(dvec<T> const& d) {
    std::vector<T> h(d.size());
    hpx::parallel::copy(ex::par, d.begin(), d.end(), h.begin());
    return h;
}
template <typename T>
void from_host(std::vector<T> const& h, dvec<T>& d) {
    hpx::parallel::copy(ex::par, h.begin(), h.end(), d.begin());
}

int check_n_triangle(int n) { return n < 0 ? 0 : n * (n + 1) / 2; }
int check_n_const(int n, int x) { return n < 0 ? 0 : n * x; }

// exclusive_scan_validate.cpp: ARRAY_SIZE 10000, INITIAL_VAL 50, FILL_VALUE 10
template <typename Policy>
void test_exclusive_scan_validate(Policy p, hip::default_executor const& exec, bool in_place) {
    int const size = 10000, init = 50, fill = 10;
    hip::allocator<int> alloc(exec.target());
    for (int variant = 0; variant < 3; ++variant) {
        std::vector<int> a;
        if (variant == 0) for (int i = 0; i < size; ++i) a.push_back(i);
        if (variant == 1) for (int i = 1; i < size; ++i) a.push_back(i);
        if (variant == 2) a.assign(size, fill);
        dvec<int> da(a.size(), alloc), db(a.size(), alloc);
        from_host(a, da);
        auto& out = in_place ? da : db;
        auto r = hpx::parallel::exclusive_scan(p, da.begin(), da.end(), out.begin(), init, std::plus<int>());
        if constexpr (!ex::is_async_execution_policy<Policy>::value) HPX_TEST(r == out.end());
        else HPX_TEST(r.get() == out.end());
        auto b = to_host(out);
        for (int i = 0; i < int(b.size()); ++i) {
            int expect = variant == 0 ? init + check_n_triangle(i - 1)
                       : variant == 1 ? init + check_n_triangle(i)
                                      : init + check_n_const(i, fill);
            if (!HPX_TEST_EQ(b[i], expect)) break;
        }
    }
}

void test_inclusive_scan_known(hip::default_executor const& exec) {
    hip::allocator<double> alloc(exec.target());
    // N x 1.0: every partial sum is an exactly representable integer
    std::size_t const n = std::size_t(1) << 26;
    dvec<double> a(n, 1.0, alloc), b(n, alloc);
    hpx::parallel::inclusive_scan(ex::par.on(exec), a.begin(), a.end(), b.begin(), 0.0, std::plus<double>());
    HPX_TEST_EQ(double(b[0]), 1.0);
    HPX_TEST_EQ(double(b[n / 2 - 1]), double(n / 2));
    HPX_TEST_EQ(double(b[n - 1]), double(n));
    auto hb = to_host(b);
    for (std::size_t i = 0; i < n; i += 4099)
        if (!HPX_TEST_EQ(hb[i], double(i + 1))) break;

    // 10007 x size_t(1), no-init overload (init = value_type())
    hip::allocator<uint64_t> ua(exec.target());
    dvec<uint64_t> c(10007, uint64_t(1), ua), d(10007, ua);
    hpx::parallel::inclusive_scan(ex::par.on(exec), c.begin(), c.end(), d.begin());
    auto hd = to_host(d);
    for (std::size_t i = 0; i < hd.size(); ++i)
        if (!HPX_TEST_EQ(hd[i], uint64_t(i + 1))) break;

    // (op, init) and (init, op) overloads agree; multiplies over small values
    std::vector<int64_t> h(777);
    for (auto& x : h) x = int64_t(gen() % 3) + 1;
    hip::allocator<int64_t> ia(exec.target());
    dvec<int64_t> e(h.size(), ia), f(h.size(), ia), g(h.size(), ia);
    from_host(h, e);
    hpx::parallel::inclusive_scan(ex::par.on(exec), e.begin(), e.end(), f.begin(), std::plus<int64_t>(), int64_t(5));
    hpx::parallel::inclusive_scan(ex::par.on(exec), e.begin(), e.end(), g.begin(), int64_t(5), std::plus<int64_t>());
    std::vector<int64_t> ref(h.size());
    int64_t acc = 5;
    for (std::size_t i = 0; i < h.size(); ++i) ref[i] = acc += h[i];
    HPX_TEST(to_host(f) == ref);
    HPX_TEST(to_host(g) == ref);
    // transform_inclusive_scan: running sum of squares
    hpx::parallel::transform_inclusive_scan(ex::par.on(exec), e.begin(), e.end(), f.begin(), std::plus<int64_t>(),
                                            fn::square{}, int64_t(0));
    acc = 0;
    for (std::size_t i = 0; i < h.size(); ++i) ref[i] = acc += h[i] * h[i];
    HPX_TEST(to_host(f) == ref);
    // transform_exclusive_scan
    hpx::parallel::transform_exclusive_scan(ex::par.on(exec), e.begin(), e.end(), f.begin(), int64_t(-3),
                                            std::plus<int64_t>(), fn::square{});
    acc = -3;
    for (std::size_t i = 0; i < h.size(); ++i) {
        ref[i] = acc;
        acc += h[i] * h[i];
    }
    HPX_TEST(to_host(f) == ref);
}

// copyif_random.cpp: half the values >= 0, half < 0, predicate !(i < 0)
void test_copy_if(hip::default_executor const& exec) {
    for (std::size_t n : {std::size_t(0), std::size_t(1), std::size_t(10007), std::size_t(5000000)}) {
        std::vector<int> h(n);
        std::uniform_int_distribution<int> pos(0, 1 << 30), neg(-(1 << 30), -1);
        for (std::size_t i = 0; i < n; ++i) h[i] = (i < n / 2) ? pos(gen) : neg(gen);
        std::shuffle(h.begin(), h.end(), gen);
        hip::allocator<int> alloc(exec.target());
        dvec<int> a(n, alloc), b(n, alloc);
        from_host(h, a);
        auto r = hpx::parallel::copy_if(ex::par.on(exec), a.begin(), a.end(), b.begin(), fn::not_less_than<int>{0});
        std::vector<int> ref;
        std::copy_if(h.begin(), h.end(), std::back_inserter(ref), [](int i) { return !(i < 0); });
        HPX_TEST(r.in() == a.end());
        HPX_TEST_EQ(std::size_t(r.out() - b.begin()), ref.size());
        auto hb = to_host(b);
        hb.resize(ref.size());
        HPX_TEST(hb == ref);  // stable: same order as the input
    }
}

// partitioned_vector_reduce.cpp: 10007 ones + init 1 = 10008
void test_reduce(hip::default_executor const& exec) {
    hip::allocator<int> ia(exec.target());
    dvec<int> a(10007, 1, ia);
    HPX_TEST_EQ(hpx::parallel::reduce(ex::par.on(exec), a.begin(), a.end(), 1), 10008);
    HPX_TEST_EQ(hpx::parallel::reduce(ex::seq, a.begin(), a.end(), 1, std::plus<int>()), 10008);
    hip::allocator<double> da(exec.target());
    dvec<double> b(10007, 1.0, da);
    HPX_TEST_EQ(hpx::parallel::reduce(ex::par.on(exec), b.begin(), b.end(), 1.0), 10008.0);
    HPX_TEST_EQ(hpx::parallel::reduce(ex::par.on(exec), b.begin(), b.end()), 10007.0);
    // empty range returns init
    HPX_TEST_EQ(hpx::parallel::reduce(ex::par.on(exec), b.begin(), b.begin(), 4.5), 4.5);

    // min / max / xor over random int64 vs std
    std::size_t const n = 3000017;
    std::vector<int64_t> h(n);
    for (auto& x : h) x = int64_t(gen());
    hip::allocator<int64_t> la(exec.target());
    dvec<int64_t> c(n, la);
    from_host(h, c);
    HPX_TEST_EQ(hpx::parallel::reduce(ex::par.on(exec), c.begin(), c.end(), INT64_MAX, fn::minimum{}),
                *std::min_element(h.begin(), h.end()));
    HPX_TEST_EQ(hpx::parallel::reduce(ex::par.on(exec), c.begin(), c.end(), INT64_MIN, fn::maximum{}),
                *std::max_element(h.begin(), h.end()));
    int64_t x = 0;
    for (auto v : h) x ^= v;
    HPX_TEST_EQ(hpx::parallel::reduce(ex::par.on(exec), c.begin(), c.end(), int64_t(0), std::bit_xor<int64_t>()), x);
    uint64_t wrap = 0;
    for (auto v : h) wrap += uint64_t(v);
    HPX_TEST_EQ(uint64_t(hpx::parallel::reduce(ex::par.on(exec), c.begin(), c.end(), int64_t(0))), wrap);

    // int32 inputs widened into an int64 accumulator (T = init's type)
    std::vector<int> hi(n);
    for (auto& v : hi) v = int(gen() % 2000001) - 1000000;
    dvec<int> d(n, ia);
    from_host(hi, d);
    int64_t s = 0;
    for (auto v : hi) s += v;
    HPX_TEST_EQ(hpx::parallel::reduce(ex::par.on(exec), d.begin(), d.end(), int64_t(0)), s);

    // transform_reduce: sum of squares; inner product (transform_reduce_binary.hpp:323)
    std::vector<int64_t> hs(100003);
    std::iota(hs.begin(), hs.end(), int64_t(-50000));
    dvec<int64_t> e(hs.size(), la), f(hs.size(), la);
    from_host(hs, e);
    from_host(hs, f);
    int64_t sq = 0;
    for (auto v : hs) sq += v * v;
    HPX_TEST_EQ(hpx::parallel::transform_reduce(ex::par.on(exec), e.begin(), e.end(), int64_t(0),
                                                std::plus<int64_t>(), fn::square{}),
                sq);
    HPX_TEST_EQ(hpx::parallel::transform_reduce(ex::par.on(exec), e.begin(), e.end(), f.begin(), int64_t(7)),
                sq + 7);
    HPX_TEST_EQ(hpx::parallel::transform_reduce(ex::par.on(exec), e.begin(), e.end(), f.begin(), int64_t(0),
                                                std::plus<int64_t>(), std::multiplies<int64_t>()),
                sq);
}

template <typename T>
void test_sort_type(hip::default_executor const& exec, std::size_t n) {
    std::vector<T> h(n);
    for (auto& x : h) {
        if constexpr (std::is_floating_point<T>::value) x = T(std::uniform_real_distribution<double>(-1e6, 1e6)(gen));
        else x = T(gen());
    }
    hip::allocator<T> alloc(exec.target());
    dvec<T> d(n, alloc);
    from_host(h, d);
    auto r = hpx::parallel::sort(ex::par.on(exec), d.begin(), d.end());
    HPX_TEST(r == d.end());
    auto ref = h;
    std::sort(ref.begin(), ref.end());
    HPX_TEST(to_host(d) == ref);
    // descending (std::greater)
    from_host(h, d);
    hpx::parallel::sort(ex::par.on(exec), d.begin(), d.end(), std::greater<T>());
    std::sort(ref.begin(), ref.end(), std::greater<T>());
    HPX_TEST(to_host(d) == ref);
}

void test_sort(hip::default_executor const& exec) {
    for (std::size_t n : {std::size_t(0), std::size_t(1), std::size_t(2), std::size_t(10007), std::size_t(3000017)}) {
        test_sort_type<uint32_t>(exec, n);
        test_sort_type<int32_t>(exec, n);
        test_sort_type<uint64_t>(exec, n);
        test_sort_type<int64_t>(exec, n);
        test_sort_type<float>(exec, n);
        test_sort_type<double>(exec, n);
    }
    // sort_by_key: stable -- equal keys keep their value order
    std::size_t const n = 1000003;
    std::vector<uint32_t> keys(n), vals(n);
    for (std::size_t i = 0; i < n; ++i) {
        keys[i] = uint32_t(gen() % 1000);
        vals[i] = uint32_t(i);
    }
    hip::allocator<uint32_t> alloc(exec.target());
    dvec<uint32_t> dk(n, alloc), dv(n, alloc);
    from_host(keys, dk);
    from_host(vals, dv);
    auto r = hpx::parallel::sort_by_key(ex::par.on(exec), dk.begin(), dk.end(), dv.begin());
    HPX_TEST(r.in1() == dk.end());
    HPX_TEST(r.in2() == dv.end());
    std::vector<std::size_t> idx(n);
    std::iota(idx.begin(), idx.end(), std::size_t(0));
    std::stable_sort(idx.begin(), idx.end(), [&](std::size_t a, std::size_t b) { return keys[a] < keys[b]; });
    auto hk = to_host(dk), hv = to_host(dv);
    bool ok = true;
    for (std::size_t i = 0; i < n && ok; ++i) ok = hk[i] == keys[idx[i]] && hv[i] == vals[idx[i]];
    HPX_TEST(ok);
}

// container_algorithms/sort.hpp:102 (sort_range_tests.hpp test_sort1/2:
// HPX_SORT_TEST_SIZE random values, default and std::greater, sync and task
// policies) and is_sorted.hpp:40-120.  5,000,000 u64 keys take the hybrid
// radix path (>= 2^22 keys).
void test_sort_range_is_sorted(hip::default_executor const& exec) {
    std::size_t const n = 5000000;
    std::vector<uint64_t> h(n);
    for (auto& x : h) x = gen();
    hip::allocator<uint64_t> alloc(exec.target());
    dvec<uint64_t> d(n, alloc);
    from_host(h, d);
    HPX_TEST(!hpx::parallel::is_sorted(ex::par.on(exec), d.begin(), d.end()));
    auto r = hpx::parallel::sort(ex::par.on(exec), d);
    HPX_TEST(r == d.end());
    auto ref = h;
    std::sort(ref.begin(), ref.end());
    HPX_TEST(to_host(d) == ref);
    HPX_TEST(hpx::parallel::is_sorted(ex::par.on(exec), d.begin(), d.end()));
    HPX_TEST(!hpx::parallel::is_sorted(ex::par.on(exec), d.begin(), d.end(), std::greater<uint64_t>()));
    hpx::parallel::sort(ex::par(ex::task).on(exec), d, std::greater<uint64_t>()).get();
    std::sort(ref.begin(), ref.end(), std::greater<uint64_t>());
    HPX_TEST(to_host(d) == ref);
    HPX_TEST(hpx::parallel::is_sorted(ex::par(ex::task).on(exec), d.begin(), d.end(), std::greater<uint64_t>()).get());
    // empty, one element, one pair out of order
    HPX_TEST(hpx::parallel::is_sorted(ex::par.on(exec), d.begin(), d.begin()));
    HPX_TEST(hpx::parallel::is_sorted(ex::par.on(exec), d.begin(), d.begin() + 1));
    std::vector<int32_t> small = {1, 2, 3, 5, 4, 6};
    hip::allocator<int32_t> ai(exec.target());
    dvec<int32_t> ds(small.size(), ai);
    from_host(small, ds);
    HPX_TEST(hpx::parallel::is_sorted(ex::par.on(exec), ds.begin(), ds.begin() + 4));
    HPX_TEST(!hpx::parallel::is_sorted(ex::par.on(exec), ds.begin(), ds.end()));
}

void test_elementwise(hip::default_executor const& exec) {
    hip::allocator<float> alloc(exec.target());
    dvec<float> a(1001, alloc), b(1001, alloc);
    hpx::parallel::fill(ex::par.on(exec), a.begin(), a.end(), 2.0f);
    auto it = hpx::parallel::fill_n(ex::par.on(exec), a.begin(), 10, -1.0f);
    HPX_TEST(it == a.begin() + 10);
    auto e = hpx::parallel::for_each_n(ex::par.on(exec), a.begin() + 10, 991, fn::affine<float>{3.0f, 1.0f});
    HPX_TEST(e == a.end());
    auto c = hpx::parallel::copy_n(ex::par.on(exec), a.begin(), 1001, b.begin());
    HPX_TEST(c.out() == b.end());
    auto hb = to_host(b);
    HPX_TEST_EQ(hb[0], -1.0f);
    HPX_TEST_EQ(hb[9], -1.0f);
    HPX_TEST_EQ(hb[10], 7.0f);
    HPX_TEST_EQ(hb[1000], 7.0f);
    // unary transform with the reference STREAM's scale step; 4-iterator binary transform
    hpx::parallel::transform(ex::par.on(exec), a.begin(), a.end(), b.begin(), fn::multiply_step<float>{0.5f});
    HPX_TEST_EQ(float(b[500]), 3.5f);
    auto t = hpx::parallel::transform(ex::par.on(exec), a.begin(), a.end(), b.begin(), b.begin() + 100, a.begin(),
                                      fn::add_step{});
    HPX_TEST(t.out() == a.begin() + 100);
    HPX_TEST_EQ(float(a[50]), 10.5f);
    HPX_TEST_EQ(float(a[100]), 7.0f);
}

int hpx_main(int argc, char* argv[]) {
    unsigned long seed = argc > 1 ? std::strtoul(argv[1], nullptr, 10) : std::random_device{}();
    std::cout << "using seed: " << seed << std::endl;
    gen.seed(seed);
    hip::target target;
    hip::default_executor exec(target);

    test_exclusive_scan_validate(ex::par.on(exec), exec, false);
    test_exclusive_scan_validate(ex::par.on(exec), exec, true);
    test_exclusive_scan_validate(ex::par(ex::task).on(exec), exec, false);
    test_exclusive_scan_validate(ex::seq, exec, true);
    test_inclusive_scan_known(exec);
    test_copy_if(exec);
    test_reduce(exec);
    test_sort(exec);
    test_sort_range_is_sorted(exec);
    test_elementwise(exec);
    return hpx::finalize();
}

int main(int argc, char* argv[]) {
    HPX_TEST_EQ(hpx::init(argc, argv), 0);
    int errors = hpx::util::report_errors();
    if (!errors) std::cout << "algorithms_known_answer: all tests passed" << std::endl;
    return errors;
}
