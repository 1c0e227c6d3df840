// Microbenchmark: the hybrid sort's LDS-resident segment sort (k_bucket_sort,
// hpx_amd/csrc/sort_kernel.hpp) over 2^30 uint64 keys in 65536 segments of
// 16384 keys (one bucket each: the bench's shape): random low 48 bits (the
// MSD levels) and low bits confined to 24 (the stable fallback path).
// build: hipcc -O3 --offload-arch=gfx950 -std=c++17 bucket.hip -o bucket
#include "../../hpx_amd/csrc/sort_kernel.hpp"

#include <algorithm>
#include <cstdio>
#include <vector>

using namespace hpxhip;
using namespace hpxhip::sort_detail;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

// key i: top 16 bits = segment (i / 16384), low 48 bits random
__global__ void k_fill(uint64_t* k, uint64_t n, uint64_t lowmask, int segbits = 14, int topbit = 48) {
    const uint64_t i = blockIdx.x * 256ull + threadIdx.x;
    if (i >= n) return;
    uint64_t z = (i ^ 0x5EEDull) + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    k[i] = ((i >> segbits) << topbit) | ((z ^ (z >> 31)) & lowmask);
}
__global__ void k_check(const uint64_t* k, uint64_t n, unsigned long long* bad) {
    const uint64_t i = blockIdx.x * 256ull + threadIdx.x;
    if (i == 0 || i >= n) return;
    if (k[i - 1] > k[i]) atomicAdd(bad, 1ull);
}

static hipEvent_t e0, e1;
template <typename F>
float bench(const char* name, F f, double keys) {
    f();
    CK(hipDeviceSynchronize());
    std::vector<float> t;
    for (int r = 0; r < 5; ++r) {
        CK(hipEventRecord(e0));
        f();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    printf("%-40s min %7.3f ms med %7.3f ms  %7.1f GB/s (16 B/key)\n", name, t[0], t[2], 16 * keys / t[0] / 1e6);
    fflush(stdout);
    return t[0];
}

template <int T, int I, int LV = 16>
void run(uint64_t* k, uint64_t* seg, uint64_t n, uint64_t mask, const char* tag) {
    // every rep sorts freshly generated keys (a re-sort of sorted segments
    // is cheaper: fewer LDS bank conflicts, odd-even rounds settle at once);
    // the fill alone is timed and subtracted
    const unsigned nseg = static_cast<unsigned>(n / 16384);
    char name[96];
    snprintf(name, sizeof name, "%s T%d I%d OE%d", tag, T, I, LV);
    const float fill = bench("  (fill only)", [&] { hipLaunchKernelGGL(k_fill, dim3(n / 256), dim3(256), 0, 0, k, n, mask); },
                             double(n));
    const float both = bench(name, [&] {
        hipLaunchKernelGGL(k_fill, dim3(n / 256), dim3(256), 0, 0, k, n, mask);
        hipLaunchKernelGGL((k_bucket_sort<uint64_t, ordered_bits<uint64_t, false>, T, I, LV>), dim3(nseg), dim3(T), 0, 0, k,
                           seg, 48, ordered_bits<uint64_t, false>{});
    }, double(n));
    printf("%-56s %7.3f ms (fill subtracted)  %7.1f GB/s (16 B/key)\n", name, both - fill, 16.0 * n / (both - fill) / 1e6);
}

// 2^30 keys in 131072 segments of 8192 (17-bit prefix, one bucket each)
template <int T, int I>
void run_small(uint64_t* k, uint64_t* seg, uint64_t n, const char* tag) {
    const unsigned nseg = static_cast<unsigned>(n / 8192);
    const uint64_t m47 = (1ull << 47) - 1;
    char name[96];
    snprintf(name, sizeof name, "%s T%d I%d", tag, T, I);
    const float fill = bench("  (fill only)", [&] { hipLaunchKernelGGL(k_fill, dim3(n / 256), dim3(256), 0, 0, k, n, m47, 13, 47); },
                             double(n));
    const float both = bench(name, [&] {
        hipLaunchKernelGGL(k_fill, dim3(n / 256), dim3(256), 0, 0, k, n, m47, 13, 47);
        hipLaunchKernelGGL((k_bucket_sort<uint64_t, ordered_bits<uint64_t, false>, T, I>), dim3(nseg), dim3(T), 0, 0, k,
                           seg, 47, ordered_bits<uint64_t, false>{});
    }, double(n));
    printf("%-56s %7.3f ms (fill subtracted)  %7.1f GB/s (16 B/key)\n", name, both - fill, 16.0 * n / (both - fill) / 1e6);
}

int main() {
    const uint64_t n = 1ull << 30;
    uint64_t *k, *seg;
    unsigned long long* bad;
    CK(hipMalloc(&k, n * 8));
    const unsigned nseg = n / 16384;
    std::vector<uint64_t> hs(2 * nseg);
    for (unsigned s = 0; s < nseg; ++s) { hs[2 * s] = uint64_t(s) * 16384; hs[2 * s + 1] = uint64_t(s + 1) * 16384; }
    CK(hipMalloc(&seg, hs.size() * 8));
    CK(hipMemcpy(seg, hs.data(), hs.size() * 8, hipMemcpyHostToDevice));
    CK(hipMalloc(&bad, 8));
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const uint64_t m48 = (1ull << 48) - 1, m24 = (1ull << 24) - 1;
    run<1024, 18, -1>(k, seg, n, m48, "segment sort, random low 48 bits (2 passes only)");
    run<1024, 18>(k, seg, n, m48, "segment sort, random low 48 bits");
    run<1024, 18>(k, seg, n, m24, "segment sort, low 24 bits (fallback)");
    {
        std::vector<uint64_t> hs2(2 * (n / 8192));
        for (uint64_t s2 = 0; s2 < n / 8192; ++s2) { hs2[2 * s2] = s2 * 8192; hs2[2 * s2 + 1] = (s2 + 1) * 8192; }
        uint64_t* seg2;
        CK(hipMalloc(&seg2, hs2.size() * 8));
        CK(hipMemcpy(seg2, hs2.data(), hs2.size() * 8, hipMemcpyHostToDevice));
        run_small<512, 18>(k, seg2, n, "segment sort 8192-key segments, 2/CU");
        CK(hipMemset(bad, 0, 8));
        hipLaunchKernelGGL(k_check, dim3(n / 256), dim3(256), 0, 0, k, n, bad);
        unsigned long long hb = 0;
        CK(hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost));
        printf("unsorted pairs after the 8192-key segment sorts: %llu\n", hb);
    }
    CK(hipMemset(bad, 0, 8));
    for (uint64_t mask : {m48, m24}) {
        CK(hipMemset(bad, 0, 8));
        hipLaunchKernelGGL(k_fill, dim3(n / 256), dim3(256), 0, 0, k, n, mask);
        hipLaunchKernelGGL((k_bucket_sort<uint64_t, ordered_bits<uint64_t, false>, 1024, 18>), dim3(nseg), dim3(1024), 0,
                           0, k, seg, 48, ordered_bits<uint64_t, false>{});
        hipLaunchKernelGGL(k_check, dim3(n / 256), dim3(256), 0, 0, k, n, bad);
        unsigned long long hb = 0;
        CK(hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost));
        printf("unsorted pairs after one segment sort (low mask %llx): %llu\n", (unsigned long long)mask, hb);
    }
    return 0;
}
