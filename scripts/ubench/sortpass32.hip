// Microbenchmark: one onesweep pass (digit 0) over 2^30 uint32 keys at several
// tile shapes (the shipped 512 x 16 u64 shape holds only 32 KiB of u32 keys).
// build: hipcc -O3 --offload-arch=gfx950 -std=c++17 sortpass32.hip -o sortpass32
#include "../../hpx_amd/csrc/sort_kernel.hpp"

#include <algorithm>
#include <cstdio>
#include <vector>

using namespace hpxhip;
using namespace hpxhip::sort_detail;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

__global__ void k_fill_rand(uint32_t* k, uint64_t n) {
    const uint64_t i = blockIdx.x * 256ull + threadIdx.x;
    if (i >= n) return;
    uint64_t z = (i ^ 0x5EEDull) + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    k[i] = static_cast<uint32_t>(z ^ (z >> 31));
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
    printf("%-40s min %7.3f ms med %7.3f ms  %6.2f Gkeys/s  %7.1f GB/s (8 B/key)\n", name, t[0], t[3],
           keys / t[0] / 1e6, 8 * keys / t[0] / 1e6);
    fflush(stdout);
}

int main() {
    const uint64_t n = 1ull << 30;
    uint32_t *kin, *kout, *counter, *err;
    unsigned long long *hist, *start, *bits;
    void* lb;
    CK(hipMalloc(&kin, n * 4));
    CK(hipMalloc(&kout, n * 4));
    CK(hipMalloc(&hist, 4 * 256 * 8));
    CK(hipMalloc(&start, 4 * 256 * 8));
    CK(hipMalloc(&bits, 256));
    CK(hipMalloc(&counter, 256));
    CK(hipMalloc(&err, 64));
    CK(hipMalloc(&lb, (n / 2048 + 1) * 256 * 4));
    CK(hipMemset(err, 0, 64));
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    hipLaunchKernelGGL(k_fill_rand, dim3(n / 256), dim3(256), 0, 0, kin, n);
    using X = ordered_bits<uint32_t, false>;
    CK(hipMemset(hist, 0, 4 * 256 * 8));
    hipLaunchKernelGGL((k_hist<uint32_t, X, 256, 4>), dim3(1024), dim3(256), 0, 0, kin, n, 0, 4, X{}, hist, bits, -1,
                       nullptr);
    hipLaunchKernelGGL(k_bin_offsets<256>, dim3(4), dim3(256), 0, 0, hist, start);
    CK(hipDeviceSynchronize());
#define PASS(T, I)                                                                                           \
    bench("u32 onesweep T" #T " I" #I, [&] {                                                                 \
        constexpr uint64_t tile = T * I;                                                                     \
        const uint64_t ntiles = (n + tile - 1) / tile;                                                       \
        CK(hipMemsetAsync(counter, 0, 256));                                                                 \
        CK(hipMemsetAsync(lb, 0, ntiles * 256 * 4));                                                         \
        hipLaunchKernelGGL((k_onesweep<uint32_t, uint32_t, false, uint32_t, X, T, I, 4>), dim3(ntiles), dim3(T), \
                           0, 0, kin, kout, (const uint32_t*)nullptr, (uint32_t*)nullptr, n, 0, start,        \
                           (uint32_t*)lb, counter, err, X{});                                               \
    }, n)
    for (int rep = 0; rep < 2; ++rep) {
        PASS(512, 16);
        PASS(512, 24);
        PASS(512, 32);
        PASS(1024, 16);
        PASS(256, 32);
    }
    uint32_t herr;
    CK(hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost));
    printf("deverr %u\n", herr);
    return 0;
}
