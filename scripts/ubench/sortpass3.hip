// Microbenchmark (round 3): look-back width of the hybrid sort's two prefix
// passes (the 9-bit field under the top byte and the top byte), shipped tile
// (512 x 16 keys, tile ids from the counter) over 2^30 random uint64 keys:
// LBB = predecessor granules each digit's thread loads per look-back step.
// The 9-bit pass fetches 1.23x its algorithmic bytes with LBB = 4
// (profiles/r03_pmc_sort.txt); fewer granules per step trade traffic for
// round trips.
// build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -I../../include sortpass3.hip -o sortpass3
#include <hpxhip/kernels/sort_kernel.hpp>

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
    printf("%-36s min %7.3f ms med %7.3f ms  %7.1f GB/s (16 B/key)\n", name, t[0], t[3], 16 * keys / t[0] / 1e6);
    fflush(stdout);
}

int main() {
    const uint64_t n = 1ull << 30;
    uint64_t *kin, *kout;
    unsigned long long *hist, *start, *bits, *xhist, *xstart;
    uint32_t *counter, *err;
    void* lb;
    CK(hipMalloc(&kin, n * 8));
    CK(hipMalloc(&kout, n * 8));
    CK(hipMalloc(&hist, 8 * 256 * 8));
    CK(hipMalloc(&start, 8 * 256 * 8));
    CK(hipMalloc(&xhist, 512 * 8));
    CK(hipMalloc(&xstart, 512 * 8));
    CK(hipMalloc(&bits, 256));
    CK(hipMalloc(&err, 64));
    const uint64_t ntiles = (n + 8191) / 8192;
    CK(hipMalloc(&lb, 256 + ntiles * 512 * 4));
    counter = static_cast<uint32_t*>(lb);
    CK(hipMemset(err, 0, 64));
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    hipLaunchKernelGGL(k_fill_rand, dim3(n / 256), dim3(256), 0, 0, kin, n);
    using X = ordered_bits<uint64_t, false>;
    CK(hipMemset(hist, 0, 8 * 256 * 8));
    CK(hipMemset(xhist, 0, 512 * 8));
    hipLaunchKernelGGL((k_hist<uint64_t, X, 256, 4>), dim3(1024), dim3(256), 0, 0, kin, n, 0, 8, X{}, hist, bits, 47,
                       xhist);
    hipLaunchKernelGGL(k_bin_offsets<256>, dim3(8), dim3(256), 0, 0, hist, start);
    hipLaunchKernelGGL(k_bin_offsets<512>, dim3(1), dim3(512), 0, 0, xhist, xstart);
    CK(hipDeviceSynchronize());
    uint32_t* lbg = reinterpret_cast<uint32_t*>(static_cast<char*>(lb) + 256);
#define PASS(RB, LBB, SHIFT, BS)                                                                               \
    bench("RB" #RB " LBB" #LBB, [&] {                                                                          \
        CK(hipMemsetAsync(lb, 0, 256 + ntiles * (1 << RB) * 4));                                              \
        hipLaunchKernelGGL((k_onesweep<uint64_t, uint32_t, false, uint32_t, X, 512, 16, LBB, RB, true, true>),    \
                           dim3(ntiles), dim3(512), 0, 0, kin, kout, (const uint32_t*)nullptr, (uint32_t*)nullptr, \
                           n, SHIFT, BS, lbg, counter, err, X{});                                             \
    }, n)
    for (int rep = 0; rep < 2; ++rep) {
        // r04: LBB 0 = no look-back at all (wrong offsets, in-bounds writes):
        // what the look-back costs each pass
        PASS(9, 0, 47, xstart);
        PASS(8, 0, 56, start + 7 * 256);
        PASS(9, 4, 47, xstart);
        PASS(9, 2, 47, xstart);
        PASS(9, 1, 47, xstart);
        PASS(9, 8, 47, xstart);
        PASS(8, 4, 56, start + 7 * 256);
        PASS(8, 2, 56, start + 7 * 256);
        PASS(8, 8, 56, start + 7 * 256);
    }
    uint32_t herr;
    CK(hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost));
    printf("deverr %u\n", herr);
    return 0;
}
