// Microbenchmark (round 5, seg9 = seg8's harness): the shipped k_bucket_sort
// (512 x 9, three workgroups per CU) against other thread / item shapes for
// ~4096-key segments: 1024 x 5 (16 waves, two per CU), 256 x 18 (four per
// CU), 768 x 6.  (seg8:) the shipped k_bucket_sort with and without
// PRE16 (the second LDS pass leaves each key's 16 sorted bits in a u16 array;
// the run detection reads 8 of them per 16-B LDS load instead of three 8-B
// keys per position).  seg6/seg7 had measured it inside a restructured copy
// of the kernel whose LDS went through a per-kernel offset table (7.9-8.7 ms
// against 5.1): this one instantiates the shipped kernel itself.  2^30 u64
// keys in 4096-key segments (segment id in the top bits, random low bits) and
// 2^30 u32 keys in 4096-key segments; the fill is timed alone and subtracted;
// sortedness checked after each shape.
// build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -I../../include seg9.hip -o seg9
#include <hpxhip/kernels/sort_kernel.hpp>

#include <algorithm>
#include <cstdio>
#include <vector>

using namespace hpxhip;
using namespace hpxhip::sort_detail;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

__global__ void k_fill(uint64_t* k, uint64_t n, int segbits, int topbit) {
    const uint64_t i = blockIdx.x * 256ull + threadIdx.x;
    if (i >= n) return;
    uint64_t z = (i ^ 0x5EEDull) + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    k[i] = ((i >> segbits) << topbit) | ((z ^ (z >> 31)) & ((1ull << topbit) - 1));
}
__global__ void k_check(const uint64_t* k, uint64_t n, unsigned long long* bad) {
    const uint64_t i = blockIdx.x * 256ull + threadIdx.x;
    if (i == 0 || i >= n) return;
    if (k[i - 1] > k[i]) atomicAdd(bad, 1ull);
}

static hipEvent_t e0, e1;
template <typename F>
float best(F f) {
    f();
    CK(hipDeviceSynchronize());
    std::vector<float> t;
    for (int r = 0; r < 7; ++r) {
        CK(hipEventRecord(e0));
        f();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    return t[0];
}

template <typename L>
void run(uint64_t* k, uint64_t n, int segbits, unsigned long long* bad, const char* tag, L launch) {
    const uint64_t S = 1ull << segbits, nseg = n / S;
    const int topbit = 64 - (30 - segbits);
    std::vector<uint64_t> hs(2 * nseg);
    for (uint64_t s = 0; s < nseg; ++s) { hs[2 * s] = s * S; hs[2 * s + 1] = (s + 1) * S; }
    uint64_t* seg;
    CK(hipMalloc(&seg, hs.size() * 8));
    CK(hipMemcpy(seg, hs.data(), hs.size() * 8, hipMemcpyHostToDevice));
    auto fill = [&] { hipLaunchKernelGGL(k_fill, dim3(n / 256), dim3(256), 0, 0, k, n, segbits, topbit); };
    const float f = best(fill);
    const float b = best([&] { fill(); launch(seg, nseg, topbit); });
    CK(hipMemset(bad, 0, 8));
    hipLaunchKernelGGL(k_check, dim3(n / 256), dim3(256), 0, 0, k, n, bad);
    unsigned long long hb = 0;
    CK(hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost));
    printf("%-52s %7.3f ms (fill %.3f subtracted)  unsorted pairs %llu\n", tag, b - f, f, hb);
    fflush(stdout);
    CK(hipFree(seg));
}

int main() {
    const uint64_t n = 1ull << 30;
    uint64_t* k;
    unsigned long long* bad;
    CK(hipMalloc(&k, n * 8));
    CK(hipMalloc(&bad, 8));
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    using X = ordered_bits<uint64_t, false>;
    for (int rep = 0; rep < 2; ++rep) {
        run(k, n, 12, bad, "shipped k_bucket_sort 512 x 9", [&](uint64_t* seg, uint64_t nseg, int top) {
            hipLaunchKernelGGL((k_bucket_sort<uint64_t, X, 512, 9, 16, uint32_t, false, false, false, 4, false>),
                               dim3(nseg), dim3(512), 0, 0, k, seg, top, X{});
        });
        run(k, n, 12, bad, "1024 x 5, MINW 2 (two per CU)", [&](uint64_t* seg, uint64_t nseg, int top) {
            hipLaunchKernelGGL((k_bucket_sort<uint64_t, X, 1024, 5, 16, uint32_t, false, false, false, 2, false>),
                               dim3(nseg), dim3(1024), 0, 0, k, seg, top, X{});
        });
        run(k, n, 12, bad, "1024 x 5, MINW 1", [&](uint64_t* seg, uint64_t nseg, int top) {
            hipLaunchKernelGGL((k_bucket_sort<uint64_t, X, 1024, 5, 16, uint32_t, false, false, false, 1, false>),
                               dim3(nseg), dim3(1024), 0, 0, k, seg, top, X{});
        });
        run(k, n, 12, bad, "256 x 18, MINW 4 (four per CU)", [&](uint64_t* seg, uint64_t nseg, int top) {
            hipLaunchKernelGGL((k_bucket_sort<uint64_t, X, 256, 18, 16, uint32_t, false, false, false, 4, false>),
                               dim3(nseg), dim3(256), 0, 0, k, seg, top, X{});
        });
        run(k, n, 12, bad, "768 x 6, MINW 2", [&](uint64_t* seg, uint64_t nseg, int top) {
            hipLaunchKernelGGL((k_bucket_sort<uint64_t, X, 768, 6, 16, uint32_t, false, false, false, 2, false>),
                               dim3(nseg), dim3(768), 0, 0, k, seg, top, X{});
        });
    }
    return 0;
}
