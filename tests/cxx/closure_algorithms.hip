// Arbitrary HPX_HOST_DEVICE callables through the non-elementwise algorithms
// of the HPX C++ layer, compiled by hipcc (include/hpx/parallel/detail/
// device_algorithms.hpp: the library's own reduce / scan / copy_if kernel
// bodies and a merge sort, instantiated with the caller's callables):
//
//   transform_reduce(policy, first, last, init, red, conv)   transform_reduce.hpp:254
//   transform_reduce(policy, first1, last1, first2, init, red, comb)  transform_reduce_binary.hpp:432
//   reduce(policy, first, last, init, op)                    reduce.hpp:200
//   inclusive_scan / exclusive_scan / transform_*_scan       inclusive_scan.hpp:288-606,
//                                                            exclusive_scan.hpp:292,
//                                                            transform_inclusive_scan.hpp:320,
//                                                            transform_exclusive_scan.hpp:317
//   copy_if(policy, first, last, dest, pred)                 copy.hpp:585
//   sort(policy, first, last, comp, proj), sort(policy, rng, comp)  sort.hpp:364,
//                                                            container_algorithms/sort.hpp:102
//
// Every result is checked against the host std:: algorithm on the same data:
// integer work exactly, the scans with a NON-commutative associative
// operator (composition of affine maps mod 2^32) so any out-of-order
// combination shows, sorts against std::stable_sort (the merge sort is
// stable; ties in input order are one valid std::sort result).
//
// usage: closure_algorithms [seed] [--big]   (--big adds 2^28-element runs)
#include <hpx/hpx.hpp>
#include <hpx/hpx_init.hpp>
#include <hpx/util/lightweight_test.hpp>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <numeric>
#include <random>
#include <vector>

namespace hip = hpx::compute::hip;
namespace ex = hpx::parallel::execution;
template <typename T>
using dvec = hpx::compute::vector<T, hip::allocator<T>>;

template <typename T>
std::vector<T> to_host(dvec<T> const& d) {
    std::vector<T> h(d.size());
    hpx::parallel::copy(ex::par, d.begin(), d.end(), h.begin());
    return h;
}
template <typename T>
dvec<T> to_dev(std::vector<T> const& h, hip::target const& t) {
    dvec<T> d(h.size(), hip::allocator<T>(t));
    hpx::parallel::copy(ex::par, h.begin(), h.end(), d.begin());
    return d;
}

// f then g, for f = (a1, b1), g = (a2, b2) packed (a << 32 | b): x -> a2 (a1 x + b1) + b2 mod 2^32
struct compose_affine {
    HPX_HOST_DEVICE uint64_t operator()(uint64_t f, uint64_t g) const {
        const uint32_t a1 = uint32_t(f >> 32), b1 = uint32_t(f), a2 = uint32_t(g >> 32), b2 = uint32_t(g);
        return (uint64_t(a2 * a1) << 32) | uint32_t(a2 * b1 + b2);
    }
};

template <typename T>
bool same(std::vector<T> const& a, std::vector<T> const& b, char const* what, std::size_t n) {
    if (a.size() != b.size()) {
        std::cout << what << " n=" << n << ": size " << a.size() << " != " << b.size() << std::endl;
        HPX_TEST(false);
        return false;
    }
    for (std::size_t i = 0; i < a.size(); ++i)
        if (a[i] != b[i]) {
            std::cout << what << " n=" << n << ": first mismatch at " << i << std::endl;
            HPX_TEST(false);
            return false;
        }
    return true;
}

void test_reductions(hip::default_executor& exec, std::mt19937_64& gen, std::size_t n) {
    auto pol = ex::par.on(exec);
    std::vector<int64_t> h(n);
    for (auto& x : h) x = int64_t(gen() % 2000001) - 1000000;
    auto d = to_dev(h, exec.target());
    // built-in red, lambda conv (plain value type)
    auto conv = [] HPX_HOST_DEVICE(int64_t x) { return (x * x) % 1009 - 3; };
    int64_t r1 = hpx::parallel::transform_reduce(pol, d.begin(), d.end(), int64_t(7), std::plus<>(), conv);
    HPX_TEST_EQ(r1, std::transform_reduce(h.begin(), h.end(), int64_t(7), std::plus<>(), conv));
    // lambda red (lifted to opt<T>), lambda conv, task policy
    auto mx = [] HPX_HOST_DEVICE(int64_t a, int64_t b) { return a < b ? b : a; };
    auto f2 = hpx::parallel::transform_reduce(ex::par(ex::task).on(exec), d.begin(), d.end(), INT64_MIN, mx,
                                              [] HPX_HOST_DEVICE(int64_t x) { return x ^ 0x5555; });
    int64_t e2 = INT64_MIN;
    for (auto x : h) e2 = std::max(e2, x ^ 0x5555);
    HPX_TEST_EQ(f2.get(), e2);
    // reduce with a lambda op on doubles holding integers (every order exact)
    std::vector<double> hd(n);
    for (std::size_t i = 0; i < n; ++i) hd[i] = double(h[i] % 4096);
    auto dd = to_dev(hd, exec.target());
    double r3 = hpx::parallel::reduce(pol, dd.begin(), dd.end(), 0.5, [] HPX_HOST_DEVICE(double a, double b) {
        return a + b;
    });
    HPX_TEST_EQ(r3, std::accumulate(hd.begin(), hd.end(), 0.5));
    // misaligned range (begin + 1) through the lifted path
    if (n > 2) {
        int64_t r4 = hpx::parallel::reduce(pol, d.begin() + 1, d.end(), int64_t(0), [] HPX_HOST_DEVICE(int64_t a, int64_t b) {
            return a + b;
        });
        HPX_TEST_EQ(r4, std::accumulate(h.begin() + 1, h.end(), int64_t(0)));
    }
    // inner product with lambdas (transform_reduce_binary.hpp:432)
    std::vector<int32_t> ha(n), hb(n);
    for (std::size_t i = 0; i < n; ++i) ha[i] = int32_t(gen() % 201) - 100, hb[i] = int32_t(gen() % 201) - 100;
    auto da = to_dev(ha, exec.target()), db = to_dev(hb, exec.target());
    auto red = [] HPX_HOST_DEVICE(int64_t a, int64_t b) { return a + b; };
    auto comb = [] HPX_HOST_DEVICE(int32_t x, int32_t y) { return int64_t(x) * y + 1; };
    int64_t r5 = hpx::parallel::transform_reduce(pol, da.begin(), da.end(), db.begin(), int64_t(0), red, comb);
    int64_t e5 = 0;
    for (std::size_t i = 0; i < n; ++i) e5 += comb(ha[i], hb[i]);
    HPX_TEST_EQ(r5, e5);
}

void test_scans(hip::default_executor& exec, std::mt19937_64& gen, std::size_t n) {
    auto pol = ex::par.on(exec);
    std::vector<uint64_t> h(n);
    for (auto& x : h) x = (uint64_t(uint32_t(gen()) | 1u) << 32) | uint32_t(gen());
    auto d = to_dev(h, exec.target());
    dvec<uint64_t> o(n + 1, hip::allocator<uint64_t>(exec.target()));
    const uint64_t init = (uint64_t(3) << 32) | 11u;
    compose_affine op;
    std::vector<uint64_t> e(n);
    // inclusive, (op, init) and (init, op) argument orders
    std::inclusive_scan(h.begin(), h.end(), e.begin(), op, init);
    hpx::parallel::inclusive_scan(pol, d.begin(), d.end(), o.begin(), op, init);
    std::vector<uint64_t> got = to_host(o);
    got.resize(n);
    same(got, e, "inclusive_scan(op, init)", n);
    hpx::parallel::inclusive_scan(ex::par(ex::task).on(exec), d.begin(), d.end(), o.begin(), init, op).get();
    got = to_host(o);
    got.resize(n);
    same(got, e, "inclusive_scan(init, op) task", n);
    // inclusive without init: the reference seeds with value_type() (inclusive_scan.hpp:526)
    std::inclusive_scan(h.begin(), h.end(), e.begin(), op, uint64_t());
    hpx::parallel::inclusive_scan(pol, d.begin(), d.end(), o.begin(), op);
    got = to_host(o);
    got.resize(n);
    same(got, e, "inclusive_scan(op)", n);
    // exclusive
    std::exclusive_scan(h.begin(), h.end(), e.begin(), init, op);
    hpx::parallel::exclusive_scan(pol, d.begin(), d.end(), o.begin(), init, op);
    got = to_host(o);
    got.resize(n);
    same(got, e, "exclusive_scan", n);
    // output offset by one element (unaligned kernel) and in place
    if (n > 1) {
        hpx::parallel::exclusive_scan(pol, d.begin(), d.end(), o.begin() + 1, init, op);
        got = to_host(o);
        same(std::vector<uint64_t>(got.begin() + 1, got.end()), e, "exclusive_scan (dest + 1)", n);
    }
    auto dcopy = to_dev(h, exec.target());
    hpx::parallel::exclusive_scan(pol, dcopy.begin(), dcopy.end(), dcopy.begin(), init, op);
    same(to_host(dcopy), e, "exclusive_scan (in place)", n);
    // transform scans: built-in op + lambda conv, lambda op + lambda conv
    std::vector<int64_t> hi(n), ei(n);
    for (auto& x : hi) x = int64_t(gen() % 1001) - 500;
    auto di = to_dev(hi, exec.target());
    dvec<int64_t> oi(n, hip::allocator<int64_t>(exec.target()));
    auto sq = [] HPX_HOST_DEVICE(int64_t x) { return x * x - 7; };
    std::transform_inclusive_scan(hi.begin(), hi.end(), ei.begin(), std::plus<>(), sq, int64_t(5));
    hpx::parallel::transform_inclusive_scan(pol, di.begin(), di.end(), oi.begin(), std::plus<>(), sq, int64_t(5));
    same(to_host(oi), ei, "transform_inclusive_scan", n);
    auto mn = [] HPX_HOST_DEVICE(int64_t a, int64_t b) { return b < a ? b : a; };
    std::transform_exclusive_scan(hi.begin(), hi.end(), ei.begin(), int64_t(1) << 40, mn, sq);
    hpx::parallel::transform_exclusive_scan(pol, di.begin(), di.end(), oi.begin(), int64_t(1) << 40, mn, sq);
    same(to_host(oi), ei, "transform_exclusive_scan", n);
    // 4-byte elements with a lambda op
    std::vector<uint32_t> h32(n), e32(n);
    for (auto& x : h32) x = uint32_t(gen());
    auto d32 = to_dev(h32, exec.target());
    dvec<uint32_t> o32(n, hip::allocator<uint32_t>(exec.target()));
    auto x2 = [] HPX_HOST_DEVICE(uint32_t a, uint32_t b) { return a ^ b; };
    std::inclusive_scan(h32.begin(), h32.end(), e32.begin(), x2, 0x1234u);
    hpx::parallel::inclusive_scan(pol, d32.begin(), d32.end(), o32.begin(), x2, 0x1234u);
    same(to_host(o32), e32, "inclusive_scan u32", n);
}

void test_copy_if(hip::default_executor& exec, std::mt19937_64& gen, std::size_t n) {
    std::vector<int64_t> h(n);
    for (auto& x : h) x = int64_t(gen() % 1000003);
    auto d = to_dev(h, exec.target());
    dvec<int64_t> o(n + 1, hip::allocator<int64_t>(exec.target()));
    auto pred = [] HPX_HOST_DEVICE(int64_t x) { return x % 3 == 1; };
    std::vector<int64_t> e;
    std::copy_if(h.begin(), h.end(), std::back_inserter(e), pred);
    auto r = hpx::parallel::copy_if(ex::par.on(exec), d.begin(), d.end(), o.begin(), pred);
    HPX_TEST(r.in() == d.end());
    const std::size_t cnt = static_cast<std::size_t>(r.out() - o.begin());
    std::vector<int64_t> got = to_host(o);
    got.resize(cnt);
    same(got, e, "copy_if", n);
    if (n > 1) {  // misaligned input, task policy
        e.clear();
        std::copy_if(h.begin() + 1, h.end(), std::back_inserter(e), pred);
        auto f = hpx::parallel::copy_if(ex::par(ex::task).on(exec), d.begin() + 1, d.end(), o.begin(), pred);
        auto rr = f.get();
        got = to_host(o);
        got.resize(static_cast<std::size_t>(rr.out() - o.begin()));
        same(got, e, "copy_if (begin + 1, task)", n);
    }
    // 4-byte elements
    std::vector<float> hf(n);
    for (auto& x : hf) x = float(int(gen() % 2001) - 1000) * 0.25f;
    auto df = to_dev(hf, exec.target());
    dvec<float> of(n, hip::allocator<float>(exec.target()));
    auto fp = [] HPX_HOST_DEVICE(float x) { return x < -10.0f || x > 100.0f; };
    std::vector<float> ef;
    std::copy_if(hf.begin(), hf.end(), std::back_inserter(ef), fp);
    auto rf = hpx::parallel::copy_if(ex::par.on(exec), df.begin(), df.end(), of.begin(), fp);
    std::vector<float> gf = to_host(of);
    gf.resize(static_cast<std::size_t>(rf.out() - of.begin()));
    same(gf, ef, "copy_if f32", n);
}

void test_sorts(hip::default_executor& exec, std::mt19937_64& gen, std::size_t n) {
    auto pol = ex::par.on(exec);
    std::vector<uint64_t> h(n);
    for (auto& x : h) x = gen();
    auto d = to_dev(h, exec.target());
    // comparator on the low 16 bits: many ties, the stable order is the check
    auto low = [] HPX_HOST_DEVICE(uint64_t a, uint64_t b) { return (a & 0xffff) < (b & 0xffff); };
    std::vector<uint64_t> e = h;
    std::stable_sort(e.begin(), e.end(), low);
    auto it = hpx::parallel::sort(pol, d.begin(), d.end(), low);
    HPX_TEST(it == d.end());
    same(to_host(d), e, "sort(comp)", n);
    // std::greater with a projection (|x|) on doubles, task policy
    std::vector<double> hd(n);
    for (auto& x : hd) x = double(int64_t(gen() % 20001) - 10000) / 8.0;
    auto dd = to_dev(hd, exec.target());
    auto absproj = [] HPX_HOST_DEVICE(double x) { return x < 0 ? -x : x; };
    std::vector<double> ed = hd;
    std::stable_sort(ed.begin(), ed.end(), [&](double a, double b) { return absproj(a) > absproj(b); });
    hpx::parallel::sort(ex::par(ex::task).on(exec), dd.begin(), dd.end(), std::greater<>(), absproj).get();
    same(to_host(dd), ed, "sort(greater, proj) task", n);
    // range form with a comparator, 4-byte keys, misaligned start
    std::vector<int32_t> hi(n);
    for (auto& x : hi) x = int32_t(gen() % 100000) - 50000;
    auto di = to_dev(hi, exec.target());
    auto by_mod = [] HPX_HOST_DEVICE(int32_t a, int32_t b) { return (a % 97) < (b % 97); };
    std::vector<int32_t> ei = hi;
    std::stable_sort(ei.begin(), ei.end(), by_mod);
    hpx::parallel::sort(pol, di, by_mod);
    same(to_host(di), ei, "sort(rng, comp)", n);
    if (n > 3) {
        std::vector<int32_t> e2 = hi;
        std::stable_sort(e2.begin() + 1, e2.end(), std::greater<>());
        auto di2 = to_dev(hi, exec.target());
        hpx::parallel::sort(pol, di2.begin() + 1, di2.end(), [] HPX_HOST_DEVICE(int32_t a, int32_t b) { return a > b; });
        same(to_host(di2), e2, "sort(begin + 1, lambda greater)", n);
    }
}

// 2^28 elements: the same paths at the benchmark's scale; host checks in O(n)
void test_big(hip::default_executor& exec, std::mt19937_64& gen) {
    const std::size_t n = std::size_t(1) << 28;
    auto pol = ex::par.on(exec);
    std::vector<int64_t> h(n);
    for (auto& x : h) x = int64_t(gen() % 2000001) - 1000000;
    auto d = to_dev(h, exec.target());
    auto conv = [] HPX_HOST_DEVICE(int64_t x) { return x * 3 + 1; };
    HPX_TEST_EQ(hpx::parallel::transform_reduce(pol, d.begin(), d.end(), int64_t(0), std::plus<>(), conv),
                std::transform_reduce(h.begin(), h.end(), int64_t(0), std::plus<>(), conv));
    auto add = [] HPX_HOST_DEVICE(int64_t a, int64_t b) { return a + b; };
    HPX_TEST_EQ(hpx::parallel::reduce(pol, d.begin(), d.end(), int64_t(0), add),
                std::accumulate(h.begin(), h.end(), int64_t(0)));
    dvec<int64_t> o(n, hip::allocator<int64_t>(exec.target()));
    hpx::parallel::inclusive_scan(pol, d.begin(), d.end(), o.begin(), add, int64_t(0));
    std::vector<int64_t> e(n);
    std::inclusive_scan(h.begin(), h.end(), e.begin());
    same(to_host(o), e, "inclusive_scan 2^28 (lambda)", n);
    auto pred = [] HPX_HOST_DEVICE(int64_t x) { return (x & 7) == 3; };
    auto r = hpx::parallel::copy_if(pol, d.begin(), d.end(), o.begin(), pred);
    e.clear();
    std::copy_if(h.begin(), h.end(), std::back_inserter(e), pred);
    std::vector<int64_t> got = to_host(o);
    got.resize(static_cast<std::size_t>(r.out() - o.begin()));
    same(got, e, "copy_if 2^28 (lambda)", n);
    // sort by a lambda: sorted under comp and the same multiset (sum / xor)
    auto cmp = [] HPX_HOST_DEVICE(int64_t a, int64_t b) { return (a ^ 0x2a) < (b ^ 0x2a); };
    hpx::parallel::sort(pol, d.begin(), d.end(), cmp);
    got = to_host(d);
    bool ordered = true;
    int64_t s0 = 0, s1 = 0, x0 = 0, x1 = 0;
    for (std::size_t i = 0; i < n; ++i) {
        if (i && cmp(got[i], got[i - 1])) ordered = false;
        s0 += h[i], s1 += got[i], x0 ^= h[i], x1 ^= got[i];
    }
    HPX_TEST(ordered);
    HPX_TEST(s0 == s1 && x0 == x1);
}

int hpx_main(int argc, char* argv[]) {
    unsigned seed = argc > 1 ? unsigned(std::strtoul(argv[1], nullptr, 10)) : std::random_device{}();
    bool big = false;
    for (int i = 1; i < argc; ++i) big = big || std::strcmp(argv[i], "--big") == 0;
    std::cout << "using seed: " << seed << std::endl;
    std::mt19937_64 gen(seed);
    hip::target t;
    hip::default_executor exec(t);
    for (std::size_t n : {std::size_t(0), std::size_t(1), std::size_t(2), std::size_t(7), std::size_t(1000),
                          std::size_t(4097), std::size_t(70001), std::size_t(1) << 20, (std::size_t(1) << 21) + 13}) {
        test_reductions(exec, gen, n);
        test_scans(exec, gen, n);
        test_copy_if(exec, gen, n);
        test_sorts(exec, gen, n);
    }
    if (big) test_big(exec, gen);
    return hpx::finalize();
}

int main(int argc, char* argv[]) {
    HPX_TEST_EQ(hpx::init(argc, argv), 0);
    int errors = hpx::util::report_errors();
    if (!errors) std::cout << "closure_algorithms: all tests passed" << std::endl;
    return errors;
}
