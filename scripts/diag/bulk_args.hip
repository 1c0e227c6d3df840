// Diagnostic: default_executor bulk launches with and without bound args.
#include <hpx/hpx.hpp>
#include <cstdio>
#include <numeric>
namespace hip = hpx::compute::hip;
namespace ex = hpx::parallel::execution;
struct bulk_test { int* out; int base; HPX_HOST_DEVICE void operator()(int i) { out[i - base] = 2 * i + 1; } };
struct bulk_test_args { HPX_HOST_DEVICE void operator()(int i, int* out, int base, int add) { out[i - base] = i + add; } };
template <class V> int check(V const& out, std::vector<int> const& v, int add, int mul, const char* what) {
    std::vector<int> h(out.size());
    hpx::parallel::copy(ex::par, out.begin(), out.end(), h.begin());
    int bad = 0; for (size_t i = 0; i < v.size(); ++i) bad += h[i] != mul * v[i] + add;
    printf("%-40s bad %d (h0=%d want %d)\n", what, bad, h[0], mul * v[0] + add); return bad;
}
int main() {
    hip::target t; hip::default_executor exec(t);
    hip::allocator<int> alloc(t);
    std::vector<int> v(107); std::iota(v.begin(), v.end(), 48432);
    hpx::compute::vector<int, hip::allocator<int>> out(v.size(), -1, alloc);
    for (int rep = 0; rep < 3; ++rep) {
        hpx::parallel::fill(ex::par, out.begin(), out.end(), -1);
        ex::bulk_sync_execute(exec, bulk_test{out.data(), 48432}, v);
        check(out, v, 1, 2, "bulk_sync no-args");
        hpx::parallel::fill(ex::par, out.begin(), out.end(), -1);
        ex::bulk_sync_execute(exec, bulk_test_args{}, v, out.data(), 48432, 7);
        check(out, v, 7, 1, "bulk_sync args");
        hpx::parallel::fill(ex::par, out.begin(), out.end(), -1);
        auto fs = ex::bulk_async_execute(exec, bulk_test{out.data(), 48432}, v);
        hpx::when_all(std::move(fs)).get();
        check(out, v, 1, 2, "bulk_async no-args when_all");
        hpx::parallel::fill(ex::par, out.begin(), out.end(), -1);
        auto gs = ex::bulk_async_execute(exec, bulk_test_args{}, v, out.data(), 48432, 7);
        gs[0].get();
        check(out, v, 7, 1, "bulk_async args get");
        hpx::parallel::fill(ex::par, out.begin(), out.end(), -1);
        auto hs = ex::bulk_async_execute(exec, bulk_test_args{}, v, out.data(), 48432, 7);
        hpx::when_all(std::move(hs)).get();
        check(out, v, 7, 1, "bulk_async args when_all");
        exec.target().synchronize();
        check(out, v, 7, 1, "  ... after synchronize");
    }
    return 0;
}
