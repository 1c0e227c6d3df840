// C++ port of tests/unit/computeapi/cuda/for_loop_compute.cu:28-118 on the
// HIP backend (two targets, `for_loop_n(par.on(exec), A, N, induction(B),
// induction(C), *C = *A + 3.0 * *B)`, checked element by element against the
// host transform), plus hpx::parallel::merge (merge.hpp:476) against
// std::merge, ascending and descending, sync and task policies.
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
