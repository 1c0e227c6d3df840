// Microbenchmark (round 2, session 2): do the relative base addresses of the
// STREAM arrays matter?  With equal low-order address bits, b[i], c[i] and
// a[i] of a triad map to the same HBM channel/bank at the same moment (the
// classic STREAM array-padding effect).  Triad and copy at 2^30 doubles with
// the shipped kernel shape (64-thread blocks, one 16-B vector per thread, nt
// loads and stores), arrays placed inside one allocation at 8 GiB + delta
// strides, against three separate hipMallocs.
// build: hipcc -O3 --offload-arch=gfx950 -std=c++17 offset6.hip -o offset6
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
        for (int r = 0; r < 7; ++r) {
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
    const uint64_t pad = 64 << 10;
    // Each trial perturbs the placement with a dummy allocation, then times the
    // triad on three plain hipMallocs and on three padded ones whose arrays
    // start 0 / 4 / 8 KiB into their allocation (b, c, a).
    for (int trial = 0; trial < 14; ++trial) {
        void* dummy = nullptr;
        if (trial) CK(hipMalloc(&dummy, uint64_t(trial) * (37ull << 20)));
        char *a, *b, *c;
        CK(hipMalloc(&b, bytes));
        CK(hipMalloc(&c, bytes));
        CK(hipMalloc(&a, bytes));
        CK(hipMemset(b, 0, bytes));
        CK(hipMemset(c, 0, bytes));
        const float t_plain = bench([&] {
            hipLaunchKernelGGL(k_triad, dim3(grid), dim3(64), 0, 0, (const V*)b, (const V*)c, (V*)a, nv); });
        CK(hipFree(a)); CK(hipFree(b)); CK(hipFree(c));
        float t[2][3];
        for (int contig = 0; contig < 2; ++contig) {
            char* seg;
            if (contig) CK(hipExtMallocWithFlags((void**)&seg, 25ull << 30, hipDeviceMallocContiguous));
            else CK(hipMalloc(&seg, 25ull << 30));
            CK(hipMemset(seg, 0, 25ull << 30));
            const uint64_t st[3] = {0, 4096, (2ull << 20) + 4096};
            for (int k = 0; k < 3; ++k) {
                char* B = seg; char* C = seg + bytes + st[k]; char* A = seg + 2 * bytes + 2 * st[k];
                t[contig][k] = bench([&] {
                    hipLaunchKernelGGL(k_triad, dim3(grid), dim3(64), 0, 0, (const V*)B, (const V*)C, (V*)A, nv); });
            }
            CK(hipFree(seg));
        }
        printf("trial %2d  plain %6.3f | seg s0 %6.3f s4K %6.3f s2M+4K %6.3f | contig s0 %6.3f s4K %6.3f s2M+4K %6.3f\n",
               trial, t_plain, t[0][0], t[0][1], t[0][2], t[1][0], t[1][1], t[1][2]);
        fflush(stdout);
        if (dummy) CK(hipFree(dummy));
    }
    return 0;
}
