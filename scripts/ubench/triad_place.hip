// Microbenchmark (round 6): the STREAM triad over three
// fresh 8-GiB hipMalloc arrays, as bench.py's step runs it (k_binary shape:
// 256-thread blocks, one 16-B vector per thread per array, nt loads and
// stores), to compare a fast and a slow placement under per-L2-channel PMC
// counters (rocprofv3 --pmc TCC_EA0_RDREQ / TCC_EA0_WRREQ, one pass each).
// Prints the arrays' virtual addresses (and their offsets mod 2 MiB / 1 GiB)
// and the best / mean of 8 launches (HIP events).  A fresh process gets a
// fresh placement.
// build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -I../../include triad_place.hip -o triad_place
#include <hpxhip/kernels/common.hpp>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

using namespace hpxhip;
using VT = vec<double, 2>;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

__global__ __launch_bounds__(256) void k_triad(const VT* __restrict__ b, const VT* __restrict__ c, VT* __restrict__ a,
                                               uint64_t nv, double s) {
    const uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x;
    if (i >= nv) return;
    const VT x = ld_stream(&b[i]), y = ld_stream(&c[i]);
    VT z;
    z.v[0] = x.v[0] + y.v[0] * s;
    z.v[1] = x.v[1] + y.v[1] * s;
    st_stream(&a[i], z);
}
__global__ void k_init(VT* p, uint64_t nv, double v) {
    const uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x;
    if (i < nv) p[i] = VT{{v, v}};
}

int main(int argc, char** argv) {
    const int logn = argc > 1 ? atoi(argv[1]) : 30;
    const uint64_t n = uint64_t(1) << logn, nv = n / 2;
    VT *a, *b, *c;
    CK(hipMalloc(&a, n * 8));
    CK(hipMalloc(&b, n * 8));
    CK(hipMalloc(&c, n * 8));
    const unsigned grid = static_cast<unsigned>((nv + 255) / 256);
    hipLaunchKernelGGL(k_init, dim3(grid), dim3(256), 0, 0, b, nv, 1.0);
    hipLaunchKernelGGL(k_init, dim3(grid), dim3(256), 0, 0, c, nv, 2.0);
    hipLaunchKernelGGL(k_init, dim3(grid), dim3(256), 0, 0, a, nv, 0.0);
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float best = 1e30f, sum = 0;
    const int reps = 8;
    for (int r = 0; r < reps; ++r) {
        CK(hipEventRecord(e0, 0));
        hipLaunchKernelGGL(k_triad, dim3(grid), dim3(256), 0, 0, b, c, a, nv, 3.0);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        best = std::min(best, ms);
        sum += ms;
    }
    auto off = [](const void* p, uint64_t m) { return static_cast<unsigned long long>(reinterpret_cast<uintptr_t>(p) % m); };
    printf("a=%p b=%p c=%p | mod 2MiB %llu %llu %llu | mod 1GiB %llu %llu %llu | b-a %lld c-b %lld MiB\n", (void*)a,
           (void*)b, (void*)c, off(a, 2u << 20), off(b, 2u << 20), off(c, 2u << 20), off(a, 1u << 30), off(b, 1u << 30),
           off(c, 1u << 30), (long long)((reinterpret_cast<intptr_t>(b) - reinterpret_cast<intptr_t>(a)) >> 20),
           (long long)((reinterpret_cast<intptr_t>(c) - reinterpret_cast<intptr_t>(b)) >> 20));
    printf("triad 2^%d: best %.4f ms (%.1f GB/s) mean %.4f ms\n", logn, best, 24.0 * n / (best * 1e-3) / 1e9, sum / reps);
    CK(hipFree(a));
    CK(hipFree(b));
    CK(hipFree(c));
    return 0;
}
