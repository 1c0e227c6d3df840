// Microbenchmark (round 2, session 2): do the relative base addresses of the
// STREAM arrays matter?  With equal low-order address bits, b[i], c[i] and
// a[i] of a triad map to the same HBM channel/bank at the same moment (the
// classic STREAM array-padding effect).  Triad and copy at 2^30 doubles with
// the shipped kernel shape (64-thread blocks, one 16-B vector per thread, nt
// loads and stores), arrays placed inside one allocation at 8 GiB + delta
// strides, against three separate hipMallocs.
// build: hipcc -O3 --offload-arch=gfx950 -std=c++17 offset.hip -o offset
#include "../../hpx_amd/csrc/common.hpp"
#include <algorithm>
#include <cstdio>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
using namespace hpxhip;
using V = vec<double, 2>;

__global__ __launch_bounds__(64) void k_triad(const V* b, const V* c, V* a, uint64_t nv) {
    const uint64_t i = blockIdx.x * 64ull + threadIdx.x;
    if (i < nv) {
        const V x = ld_stream(&b[i]), y = ld_stream(&c[i]);
        V r;
        r.v[0] = x.v[0] + 3.0 * y.v[0];
        r.v[1] = x.v[1] + 3.0 * y.v[1];
        st_stream(&a[i], r);
    }
}
__global__ __launch_bounds__(64) void k_copy(const V* in, V* out, uint64_t nv) {
    const uint64_t i = blockIdx.x * 64ull + threadIdx.x;
    if (i < nv) st_stream(&out[i], ld_stream(&in[i]));
}

int main() {
    const uint64_t n = 1ull << 30, nv = n / 2, bytes = n * 8;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto bench = [&](const char* name, double model, auto f) {
        f();
        CK(hipDeviceSynchronize());
        std::vector<float> ts;
        for (int r = 0; r < 9; ++r) {
            CK(hipEventRecord(e0));
            f();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            ts.push_back(ms);
        }
        std::sort(ts.begin(), ts.end());
        printf("%-46s min %7.3f ms med %7.3f ms  %7.1f GB/s\n", name, ts[0], ts[4], model / ts[0] / 1e6);
        fflush(stdout);
    };
    const unsigned grid = unsigned(nv / 64);
    for (int pass = 0; pass < 2; ++pass) {
        {  // separate allocations (what the library does today)
            char *a, *b, *c;
            CK(hipMalloc(&a, bytes));
            CK(hipMalloc(&b, bytes));
            CK(hipMalloc(&c, bytes));
            CK(hipMemset(b, 0, bytes));
            CK(hipMemset(c, 0, bytes));
            printf("separate: a %% 2MiB = %lu, b-a = %ld, c-a = %ld\n", (unsigned long)((uintptr_t)a % (2 << 20)),
                   (long)(b - a), (long)(c - a));
            bench("triad separate hipMallocs", 24.0 * n, [&] {
                hipLaunchKernelGGL(k_triad, dim3(grid), dim3(64), 0, 0, (const V*)b, (const V*)c, (V*)a, nv); });
            bench("copy separate hipMallocs", 16.0 * n, [&] {
                hipLaunchKernelGGL(k_copy, dim3(grid), dim3(64), 0, 0, (const V*)b, (V*)a, nv); });
            CK(hipFree(a));
            CK(hipFree(b));
            CK(hipFree(c));
        }
        char* base;
        const uint64_t slack = 64ull << 20;
        CK(hipMalloc(&base, 3 * bytes + 3 * slack));
        CK(hipMemset(base, 0, 3 * bytes + 3 * slack));
        const uint64_t deltas[] = {0, 256, 4096, 8192, 65536, 1ull << 20, 3ull << 20, 17ull << 20, 2048 + 256};
        for (uint64_t d : deltas) {
            char* b = base;
            char* c = base + bytes + slack + d;
            char* a = base + 2 * (bytes + slack) + 2 * d;
            char name[96];
            snprintf(name, sizeof name, "triad one alloc, stride 8GiB+64MiB+%lu", (unsigned long)d);
            bench(name, 24.0 * n, [&] {
                hipLaunchKernelGGL(k_triad, dim3(grid), dim3(64), 0, 0, (const V*)b, (const V*)c, (V*)a, nv); });
            snprintf(name, sizeof name, "copy  one alloc, stride 8GiB+64MiB+%lu", (unsigned long)d);
            bench(name, 16.0 * n, [&] {
                hipLaunchKernelGGL(k_copy, dim3(grid), dim3(64), 0, 0, (const V*)b, (V*)c, nv); });
        }
        CK(hipFree(base));
    }
    return 0;
}
