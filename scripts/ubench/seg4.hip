// Microbenchmark (round 4): the segment sort's occupancy.  The shipped
// 17-bit form sorts ~8192-key buckets in 512-thread workgroups (72 KiB of
// LDS keys, two per CU); an 18-bit prefix would give ~4096-key buckets that
// 256-thread workgroups sort with 36 KiB of LDS, four per CU (the same 16
// waves per CU in four independent barrier domains).  2^30 u64 keys with the
// segment id in the top bits and random low bits, (begin, end) pairs; the fill
// is timed alone and subtracted; sortedness checked after each shape.
// build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -I../../include seg4.hip -o seg4
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

template <int T, int I, int MINW = 4>
void run(uint64_t* k, uint64_t n, int segbits, unsigned long long* bad, const char* tag) {
    const uint64_t S = 1ull << segbits, nseg = n / S;
    const int topbit = 64 - (30 - segbits);  // the segment id above the random bits
    std::vector<uint64_t> hs(2 * nseg);
    for (uint64_t s = 0; s < nseg; ++s) { hs[2 * s] = s * S; hs[2 * s + 1] = (s + 1) * S; }
    uint64_t* seg;
    CK(hipMalloc(&seg, hs.size() * 8));
    CK(hipMemcpy(seg, hs.data(), hs.size() * 8, hipMemcpyHostToDevice));
    auto fill = [&] { hipLaunchKernelGGL(k_fill, dim3(n / 256), dim3(256), 0, 0, k, n, segbits, topbit); };
    const float f = best(fill);
    const float b = best([&] {
        fill();
        hipLaunchKernelGGL((k_bucket_sort<uint64_t, ordered_bits<uint64_t, false>, T, I, 16, uint32_t, false, false, false, MINW>), dim3(nseg), dim3(T), 0, 0, k,
                           seg, topbit, ordered_bits<uint64_t, false>{});
    });
    CK(hipMemset(bad, 0, 8));
    hipLaunchKernelGGL(k_check, dim3(n / 256), dim3(256), 0, 0, k, n, bad);
    unsigned long long hb = 0;
    CK(hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost));
    printf("%-44s T%4d I%2d  %7.3f ms (fill %.3f subtracted)  %7.1f GB/s (16 B/key)  unsorted pairs %llu\n", tag, T,
           I, b - f, f, 16.0 * n / (b - f) / 1e6, hb);
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
    for (int rep = 0; rep < 2; ++rep) {
        run<512, 18>(k, n, 13, bad, "8192-key segments (shipped 17-bit form)");
        run<256, 18>(k, n, 12, bad, "4096-key segments, 4 per CU");
        run<512, 9>(k, n, 12, bad, "4096-key segments, 512 x 9");
        run<1024, 9, 8>(k, n, 13, bad, "8192-key segments, 1024 x 9, 2/CU");
        run<1024, 9, 4>(k, n, 13, bad, "8192-key segments, 1024 x 9, 1/CU");
        run<768, 12, 6>(k, n, 13, bad, "8192-key segments, 768 x 12, 2/CU");
        run<512, 18, 4>(k, n, 13, bad, "8192-key segments (shipped 17-bit form)");
    }
    return 0;
}
