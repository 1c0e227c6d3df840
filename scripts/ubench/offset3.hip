// Microbenchmark (round 2, session 2): do the relative base addresses of the
// STREAM arrays matter?  With equal low-order address bits, b[i], c[i] and
// a[i] of a triad map to the same HBM channel/bank at the same moment (the
// classic STREAM array-padding effect).  Triad and copy at 2^30 doubles with
// the shipped kernel shape (64-thread blocks, one 16-B vector per thread, nt
// loads and stores), arrays placed inside one allocation at 8 GiB + delta
// strides, against three separate hipMallocs.
// build: hipcc -O3 --offload-arch=gfx950 -std=c++17 offset3.hip -o offset3
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
    auto bench = [&](auto f) {
        f();
        CK(hipDeviceSynchronize());
        std::vector<float> ts;
        for (int r = 0; r < 5; ++r) {
            CK(hipEventRecord(e0));
            f();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            ts.push_back(ms);
        }
        std::sort(ts.begin(), ts.end());
        return ts[0];
    };
    const unsigned grid = unsigned(nv / 64);
    const uint64_t MB = 1ull << 20;
    char* base;
    CK(hipMalloc(&base, 3 * bytes + 1024 * MB));
    CK(hipMemset(base, 0, 3 * bytes + 1024 * MB));
    // b at 0; c at 8 GiB + kc * 2 MiB + sub; a at 16 GiB + 512 MiB + ka * 2 MiB + 2 sub
    const int kcs[] = {0, 1, 2, 3, 5, 8, 16, 64, 128, 255};
    const int kas[] = {0, 1, 3, 7, 100};
    const uint64_t subs[] = {0, 4096};
    for (uint64_t sub : subs)
        for (int kc : kcs) {
            printf("sub %5lu kc %3d:", (unsigned long)sub, kc);
            for (int ka : kas) {
                const char* B = base;
                const char* C = base + bytes + kc * 2 * MB + sub;
                char* A = base + 2 * bytes + 512 * MB + ka * 2 * MB + 2 * sub;
                const float t = bench([&] {
                    hipLaunchKernelGGL(k_triad, dim3(grid), dim3(64), 0, 0, (const V*)B, (const V*)C, (V*)A, nv); });
                printf("  ka %3d %6.3f", ka, t);
            }
            printf("\n");
            fflush(stdout);
        }
    return 0;
}
