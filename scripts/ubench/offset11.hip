// Microbenchmark (round 2, session 2): do the relative base addresses of the
// STREAM arrays matter?  With equal low-order address bits, b[i], c[i] and
// a[i] of a triad map to the same HBM channel/bank at the same moment (the
// classic STREAM array-padding effect).  Triad and copy at 2^30 doubles with
// the shipped kernel shape (64-thread blocks, one 16-B vector per thread, nt
// loads and stores), arrays placed inside one allocation at 8 GiB + delta
// strides, against three separate hipMallocs.
// build: hipcc -O3 --offload-arch=gfx950 -std=c++17 offset11.hip -o offset11
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
// R regions streamed at once: block b takes chunk (b % R) * (nb / R) + b / R,
// so with R = 8 each XCD (blocks are dealt to XCDs round robin) walks its own
// eighth of the arrays.
template <int R>
__global__ __launch_bounds__(64) void k_triad_reg(const V* b, const V* c, V* a, uint64_t nv) {
    const uint64_t nb = gridDim.x;
    const uint64_t blk = (blockIdx.x % R) * (nb / R) + blockIdx.x / R;
    const uint64_t i = blk * 64ull + threadIdx.x;
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
    const uint64_t G8 = bytes, K4 = 4096, M2 = 2ull << 20;
    struct lay { const char* name; uint64_t a, b, c; };
    const lay lays[] = {
        {"A out@0 in@8G,16G", 0, G8 + K4, 2 * G8 + 2 * K4},
        {"C out@16G in@0,8G", 2 * G8 + 2 * K4, 0, G8 + K4},
        {"E out@8G in@0,16G", G8 + K4, 0, 2 * G8 + 2 * K4},
    };
    for (int trial = 0; trial < 8; ++trial) {
        void* dummy = nullptr;
        if (trial) CK(hipMalloc(&dummy, uint64_t(trial) * (37ull << 20)));
        char* seg;
        CK(hipMalloc(&seg, 56ull << 30));
        CK(hipMemset(seg, 0, 56ull << 30));
        printf("trial %d", trial);
        for (const lay& L : lays) {
            if (std::max(L.a, std::max(L.b, L.c)) + bytes > (56ull << 30)) { printf("layout out of bounds\n"); return 1; }
            const V* B = (const V*)(seg + L.b); const V* C = (const V*)(seg + L.c); V* A = (V*)(seg + L.a);
            const float t0 = bench([&] { hipLaunchKernelGGL(k_triad, dim3(grid), dim3(64), 0, 0, B, C, A, nv); });
            const float t8 = bench([&] { hipLaunchKernelGGL(k_triad_reg<8>, dim3(grid), dim3(64), 0, 0, B, C, A, nv); });
            const float t64 = bench([&] { hipLaunchKernelGGL(k_triad_reg<64>, dim3(grid), dim3(64), 0, 0, B, C, A, nv); });
            printf(" | %s flat %6.3f reg8 %6.3f reg64 %6.3f", L.name, t0, t8, t64);
        }
        printf("\n");
        fflush(stdout);
        CK(hipFree(seg));
        if (dummy) CK(hipFree(dummy));
    }
    return 0;
}
