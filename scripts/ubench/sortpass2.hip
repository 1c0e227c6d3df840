// Microbenchmark: one LSD onesweep pass (digit 0) of the shipped kernel
// (hpx_amd/csrc/sort_kernel.hpp) over 2^30 random uint64 keys, at several
// tile shapes and look-back widths; plus the all-pass histogram.
// build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -I../../include sortpass2.hip -o sortpass2
#include "../../hpx_amd/csrc/sort_kernel.hpp"

#include <algorithm>
#include <cstdio>
#include <vector>

using namespace hpxhip;
using namespace hpxhip::sort_detail;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

__global__ void k_fill_rand(uint64_t* k, uint64_t n) {
    const uint64_t i = blockIdx.x * 256ull + threadIdx.x;
    if (i >= n) return;
    uint64_t z = (i ^ 0x5EEDull) + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    k[i] = z ^ (z >> 31);
}

static hipEvent_t e0, e1;
template <typename F>
void bench(const char* name, F f, double keys) {
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
    printf("%-36s min %7.3f ms med %7.3f ms  %6.2f Gkeys/s  %7.1f GB/s (16 B/key)\n", name, t[0], t[3],
           keys / t[0] / 1e6, 16 * keys / t[0] / 1e6);
    fflush(stdout);
}

int main() {
    const uint64_t n = 1ull << 30;
    uint64_t *kin, *kout;
    unsigned long long *hist, *start, *bits;
    uint32_t *counter, *err;
    void* lb;
    CK(hipMalloc(&kin, n * 8));
    CK(hipMalloc(&kout, n * 8));
    CK(hipMalloc(&hist, 8 * 256 * 8));
    CK(hipMalloc(&start, 8 * 256 * 8));
    CK(hipMalloc(&bits, 256));
    CK(hipMalloc(&counter, 256));
    CK(hipMalloc(&err, 64));
    const size_t lb_bytes = (n / 2048 + 1) * 256 * 4;  // >= ntiles * 256 granules for tiles >= 2048 keys
    CK(hipMalloc(&lb, lb_bytes));
    CK(hipMemset(err, 0, 64));
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    hipLaunchKernelGGL(k_fill_rand, dim3(n / 256), dim3(256), 0, 0, kin, n);
    using X = ordered_bits<uint64_t, false>;
#define HIST(C, G, FIRST)                                                                                     \
    bench("hist copies" #C " grid" #G " digits from " #FIRST, [&] {                                                          \
        CK(hipMemsetAsync(hist, 0, 8 * 256 * 8));                                                    \
        hipLaunchKernelGGL((k_hist<uint64_t, X, 256, C>), dim3(G), dim3(256), 0, 0, kin, n, FIRST, 8, X{}, hist, bits, -1, nullptr); \
    }, n / 2.0)  // 8 B/key: GB/s column = read bandwidth
    HIST(4, 1024, 0); HIST(4, 1024, 6); HIST(4, 1024, 7);
    hipLaunchKernelGGL(k_bin_offsets<256>, dim3(8), dim3(256), 0, 0, hist, start);
    CK(hipDeviceSynchronize());

#define PASS(T, I, B)                                                                                         \
    bench("onesweep T" #T " I" #I " LBB" #B, [&] {                                                           \
        constexpr uint64_t tile = T * I;                                                                     \
        const uint64_t ntiles = (n + tile - 1) / tile;                                                       \
        CK(hipMemsetAsync(counter, 0, 256));                                                                 \
        CK(hipMemsetAsync(lb, 0, ntiles * 256 * 4));                                                         \
        hipLaunchKernelGGL((k_onesweep<uint64_t, uint32_t, false, uint32_t, X, T, I, B>), dim3(ntiles), dim3(T), \
                           0, 0, kin, kout, (const uint32_t*)nullptr, (uint32_t*)nullptr, n, 0, start,        \
                           (uint32_t*)lb, counter, err, X{});                                               \
    }, n)
    // 9-bit digit [0, 9) offsets for the RB = 9 variants
    unsigned long long *xhist, *xstart;
    CK(hipMalloc(&xhist, 512 * 8));
    CK(hipMalloc(&xstart, 512 * 8));
    CK(hipMemset(xhist, 0, 512 * 8));
    CK(hipMemset(hist, 0, 8 * 256 * 8));
    hipLaunchKernelGGL((k_hist<uint64_t, X, 256, 4>), dim3(1024), dim3(256), 0, 0, kin, n, 0, 8, X{}, hist, bits, 0, xhist);
    hipLaunchKernelGGL(k_bin_offsets<256>, dim3(8), dim3(256), 0, 0, hist, start);
    hipLaunchKernelGGL(k_bin_offsets<512>, dim3(1), dim3(512), 0, 0, xhist, xstart);
    void* lb9;
    CK(hipMalloc(&lb9, (n / 8192 + 1) * 512 * 4));
#define PASSX(RB, ST, BS)                                                                                      \
    bench("onesweep T512 I16 LBB4 RB" #RB " stage " #ST, [&] {                                               \
        const uint64_t ntiles = (n + 8191) / 8192;                                                           \
        CK(hipMemsetAsync(counter, 0, 256));                                                                 \
        CK(hipMemsetAsync(lb9, 0, ntiles * (1 << RB) * 4));                                                  \
        hipLaunchKernelGGL((k_onesweep<uint64_t, uint32_t, false, uint32_t, X, 512, 16, 4, RB, ST>), dim3(ntiles), \
                           dim3(512), 0, 0, kin, kout, (const uint32_t*)nullptr, (uint32_t*)nullptr, n, 0, BS,    \
                           (uint32_t*)lb9, counter, err, X{});                                              \
    }, n)
    for (int rep = 0; rep < 2; ++rep) {
        PASSX(8, true, start);
        PASSX(8, false, start);
        PASSX(9, true, xstart);
        PASSX(9, false, xstart);
    }
    uint32_t herr;
    CK(hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost));
    printf("deverr %u\n", herr);
    return 0;
}
